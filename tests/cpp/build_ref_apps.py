"""Compile the reference's own app mains UNCHANGED against this tree's
drop-in headers (include/swiftmpi/: the reference's include names) and
libswps.so — the north star's "each app is a drop-in".

    python tests/cpp/build_ref_apps.py        (also run by __graft_entry__.build())

Sources are read where they lie under /root/reference (nothing is copied);
the binaries go to tests/cpp/_ref_apps/ (git-ignored; they travel to the GPU
box with the tree, where /root/reference does not exist, and find libswps.so
through an $ORIGIN rpath).  Test infrastructure: the product never runs them."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src/apps"
OUT = os.path.join(HERE, "_ref_apps")
APPS = {"w2v": "word2vec/w2v.cpp", "w2v_local": "word2vec/w2v_local.cpp", "lr": "logistic/lr.cpp",
        "sent2vec": "sent2vec/sent2vec.cpp"}


def command(name):
    inc = os.path.join(ROOT, "include")
    lib = os.path.join(ROOT, "swiftmpi_amd", "lib")
    # -I-: quoted includes are not looked up next to the reference source (its own headers), but
    # in include/ and include/swiftmpi/apps/word2vec — where "../../swiftmpi.h" and
    # "word2vec_global.h" / "word2vec.h" resolve to the drop-in headers
    return ["g++", "-std=c++11", "-O2", "-I-", "-I" + inc, "-I" + os.path.join(inc, "swiftmpi", "apps", "word2vec"),
            os.path.join(REF, APPS[name]), "-L" + lib, "-lswps", "-pthread",
            "-Wl,-rpath,$ORIGIN/../../../swiftmpi_amd/lib", "-o", os.path.join(OUT, name)]


def build(verbose=False):
    """Returns {name: binary path}; {} when the reference tree is absent (the GPU box)."""
    if not os.path.isdir(REF):
        return {}
    os.makedirs(OUT, exist_ok=True)
    out = {}
    for name in APPS:
        cmd = command(name)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("reference app %s does not compile against include/swiftmpi:\n%s\n%s"
                               % (name, " ".join(cmd), r.stderr[-4000:]))
        out[name] = cmd[-1]
        if verbose:
            print("built", cmd[-1])
    return out


def binaries():
    return {n: os.path.join(OUT, n) for n in APPS if os.access(os.path.join(OUT, n), os.X_OK)}


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
