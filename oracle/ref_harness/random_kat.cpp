// Known-answer harness for the reference's RNG (oracle/_ref build only).
// Compiles the reference's own utils/random.h UNMODIFIED, straight from
// /root/reference/src (random.h includes only <random>, so no stand-in header
// is needed).  Prints the first N outputs of swift_snails::Random(2008)'s main
// LCG (operator()) and of its float LCG (gen_float), as JSON.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "utils/random.h"

int main(int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1000;
  swift_snails::Random a(2008), b(2008);
  printf("{\"seed\": 2008, \"n\": %d, \"lcg\": [", n);
  for (int i = 0; i < n; i++) printf(i ? ", \"%llu\"" : "\"%llu\"", (unsigned long long)a());
  printf("], \"gen_float_bits\": [");
  for (int i = 0; i < n; i++) {
    float f = b.gen_float();
    unsigned u;
    memcpy(&u, &f, 4);
    printf(i ? ", %u" : "%u", u);
  }
  printf("]}\n");
  return 0;
}
