"""Host-side logic of libswps.so (no GPU): ABI surface and the C++ host code
against the oracle."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, zipf_corpus


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "swps.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(swps_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol(lib):
    import ctypes
    from swiftmpi_amd import capi
    L = ctypes.CDLL(capi.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) > 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(capi.PROTOS), set(syms) ^ set(capi.PROTOS)


def test_library_is_gfx950_hip():
    import subprocess
    from swiftmpi_amd import capi
    out = subprocess.run(["readelf", "-S", capi.LIB_PATH], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_hash_functions_match_oracle(lib, oracle_mod):
    rng = np.random.default_rng(0)
    keys = rng.integers(0, 2 ** 63, 1000, dtype=np.int64).astype(np.uint64)
    for k in keys[:200]:
        assert lib.fmix64(int(k)) == oracle_mod.fmix64(int(k))
    for w in ["a", "superjom", "而且", "w0", "w253853", "x\ty", "ab\r"]:
        assert lib.bkdr(w) == oracle_mod.bkdr(w)
    for frag, nodes in [(1000, 1), (1000, 2), (1000, 8), (2000, 8), (8000, 8), (7, 7)]:
        t = lib.hashfrag_table(frag, nodes)
        assert np.array_equal(t, oracle_mod.hashfrag_table(frag, nodes))
        ids = lib.to_node_id(keys, frag, t)
        ref = [oracle_mod.to_node_id(int(k), frag, t) for k in keys[:100]]
        assert ids[:100].tolist() == ref
    with pytest.raises(lib.SwpsError):
        lib.hashfrag_table(3, 8)


def test_glibc_rand_emulation(lib, oracle_mod):
    # skips of 4096+ take the polynomial jump (GlibcRand::discard), shorter ones step
    for seed, skip in [(1, 0), (1, 2), (7, 1000), (0, 5), (1, 4096), (3, 4097), (1, 1234567), (9, 30000001)]:
        assert np.array_equal(lib.glibc_rand(3000, seed, skip), oracle_mod.libc_rand(3000, seed, skip))


@pytest.mark.parametrize("seed,vocab,table", [(5, 300, 10 ** 7), (6, 1500, 10 ** 8), (8, 40, 10 ** 5)])
def test_unigram_starts_match_literal_table(lib, oracle_mod, tmp_path, seed, vocab, table):
    path = zipf_corpus(str(tmp_path / "c.txt"), 200, vocab, seed=seed)
    m = oracle_mod.W2V(path, 8, minibatch=20, table_size=table)
    keys, counts = m.vocab()
    st = lib.unigram_starts(keys, counts, table)
    assert np.array_equal(st, m.table_starts())
    idx = np.random.default_rng(seed).integers(0, table, 5000).astype(np.uint64)
    vid = np.searchsorted(st, idx, side="right") - 1
    assert np.array_equal(vid.astype(np.uint32), m.table_at(idx))


def test_config_parser(tmp_path):
    from swiftmpi_amd import Config
    sub = tmp_path / "common.conf"
    sub.write_text("[server]\nfrag_num: 1000\n")
    conf = tmp_path / "demo.conf"
    conf.write_text("import %s\n[ worker ]\n# comment\nminibatch: 5000\nminibatch: 7\nnthreads: 1\n"
                    "[word2vec]\nlen_vec: 100\nsample: 0.00001\n" % sub)
    c = Config(str(conf))
    assert c.get_int("worker", "minibatch") == 5000  # std::map::insert keeps the first
    assert c.get_int("server", "frag_num") == 1000
    assert c.get_float("word2vec", "sample") == 1e-5
    with pytest.raises(KeyError):
        c.get("cluster", "server_num")


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "swiftmpi_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dirpath, f), errors="replace").read()
                assert "import oracle" not in src and "from oracle" not in src and "swps_oracle" not in src, f


def test_library_built_from_checked_out_sources(lib):
    """Build provenance: the library in the tree (prebuilt ones travel to the
    GPU box) carries the hash of exactly the csrc/ + include/ it was built
    from; a stale library fails here instead of silently testing old code."""
    from swiftmpi_amd import build, capi
    assert capi.lib().swps_build_hash().decode() == build.source_hash()
    assert build.library_hash() == build.source_hash()
