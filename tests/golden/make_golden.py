"""Regenerate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists; the fixtures are committed so the GPU
box never needs the reference).

* lcg_seed2008.json  — first 2000 outputs of the reference's own
  swift_snails::Random(2008) (utils/random.h, compiled unmodified by
  `make -C oracle ref` into oracle/_ref/random_kat).
* lr_data.txt        — the reference's bundled dataset
  src/apps/logistic/data.txt (a data fixture, copied verbatim).
* lr_reference_quality.json — outputs of the reference binary on lr_data.txt
  recorded in SURVEY.md §6 (B=200, lr 0.05, nthreads 1, predict mode after
  the text dump; log-loss/accuracy computed from its prediction file).
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    out = subprocess.check_output([os.path.join(ROOT, "oracle", "_ref", "random_kat"), "2000"])
    data = json.loads(out)
    data["source"] = "reference utils/random.h:25-47 compiled unmodified (oracle/ref_harness/random_kat.cpp)"
    with open(os.path.join(HERE, "lcg_seed2008.json"), "w") as f:
        json.dump(data, f)
    shutil.copyfile(os.path.join(REF, "apps/logistic/data.txt"), os.path.join(HERE, "lr_data.txt"))
    q = {
        "source": "SURVEY.md §6 — reference lr.cpp binary on src/apps/logistic/data.txt, "
                  "minibatch 200, initial_learning_rate 0.05, nthreads 1, deterministic",
        "minibatch": 200, "lr": 0.05,
        "epochs": {"20": {"logloss": 0.4383, "accuracy": 0.801},
                   "100": {"logloss": 0.3357, "accuracy": 0.842}},
        "rounding": "4 significant decimals for log-loss, 3 for accuracy",
    }
    with open(os.path.join(HERE, "lr_reference_quality.json"), "w") as f:
        json.dump(q, f, indent=1)
    print("ok")


if __name__ == "__main__":
    sys.exit(main())
