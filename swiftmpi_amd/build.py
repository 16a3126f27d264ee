"""Build libswps.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m swiftmpi_amd.build [--force]

The shared library lands in swiftmpi_amd/lib/ (git-ignored, travels to the GPU
box with the repo snapshot).  Object files are cached in build/.
"""
import concurrent.futures
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJDIR = os.path.join(ROOT, "build", "swps")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libswps.so")
ARCH = os.environ.get("SWPS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: the reference's fp64 arithmetic rounds every product
# before the add (x86-64 without FMA); contracting into fma would change bits.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}", "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-result"]
LDFLAGS = ["-shared", f"--offload-arch={ARCH}", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def headers():
    """The library's own headers and the C ABI it implements (include/swps.h); the C++ drop-in
    headers over it (swiftmpi_compat.h, swiftmpi/) are not part of the library."""
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs + [os.path.join(INCLUDE, "swps.h")]


HASH_MARK = "SWPS_BUILD_HASH:"


def source_hash():
    """sha256 over every source and header the library is built from (csrc/ and include/swps.h;
    name, then content)."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(sources() + headers(), key=os.path.basename):
        h.update(os.path.basename(p).encode() + b"\0")
        h.update(open(p, "rb").read())
    return h.hexdigest()


def library_hash(path=LIB):
    """The source hash stamped into a built library (read from its bytes, no load), or None."""
    try:
        blob = open(path, "rb").read()
    except OSError:
        return None
    i = blob.find(HASH_MARK.encode())
    return blob[i + len(HASH_MARK):i + len(HASH_MARK) + 64].decode() if i >= 0 else None


def _hash_obj(digest):
    """A one-function object exporting swps_build_hash() = digest (rebuilt when the sources change)."""
    src = os.path.join(OBJDIR, "swps_build_hash.cpp")
    obj = src + ".o"
    text = ('extern "C" const char *swps_build_hash(void) {\n'
            '  static const char stamp[] = "%s%s";\n'
            '  return stamp + %d;\n}\n' % (HASH_MARK, digest, len(HASH_MARK)))
    if not os.path.exists(src) or open(src).read() != text or not os.path.exists(obj):
        with open(src, "w") as f:
            f.write(text)
        r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("build-hash object: " + r.stderr)
    return obj


def _obj(src):
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = _obj(src)
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force=False, verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sources()
    hdrs = headers()
    digest = source_hash()
    if not force and not _stale(LIB, srcs + hdrs) and library_hash() == digest:
        return LIB  # the in-tree library was built from exactly these sources (e.g. on the GPU box)
    todo = [s for s in srcs if force or _stale(_obj(s), [s] + hdrs)]
    if todo:
        workers = min(len(todo), int(os.environ.get("MAX_JOBS", "8")), 16)
        with concurrent.futures.ThreadPoolExecutor(workers) as ex:
            for obj in ex.map(_compile, todo):
                if verbose:
                    print("compiled", obj)
    objs = [_obj(s) for s in srcs] + [_hash_obj(digest)]
    if force or todo or _stale(LIB, objs) or library_hash() != digest:
        cmd = [HIPCC] + LDFLAGS + objs + ["-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("linked", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
