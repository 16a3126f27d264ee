"""The C++11 host boundary (include/swiftmpi_compat.h): the reference's
parameter-server client API and app mains compiled with g++ -std=c++11
against libswps.so (tests/cpp/compat_apps.cpp).

CPU: the header compiles as strict C++11 and the driver links.
GPU: the PS-level client (pull_with_barrier / push_with_barrier with the
app's own value codecs) applies the reference's AdaGrad exactly, and the
app-level mains reproduce the Python mirror's results on the same inputs."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, int_corpus, word_dump, zipf_corpus

W2V_CONF = """[ worker ]
minibatch: 20
nthreads: 1
[ server ]
frag_num: 1000
shard_num: 300
initial_learning_rate: 0.7
[word2vec]
len_vec: 16
min_sentence_length: 1
window: 3
learning_rate: 0.05
negative: 4
sample: 0.001
"""

LR_CONF = """[ worker ]
minibatch: 200
[ server ]
initial_learning_rate: 0.05
"""


@pytest.fixture(scope="module")
def compat_bin(lib, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cpp") / "compat_apps")
    libdir = os.path.join(ROOT, "swiftmpi_amd", "lib")
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "compat_apps.cpp"), "-L" + libdir, "-lswps", "-L/opt/rocm/lib",
           "-Wl,-rpath," + libdir, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def test_compat_header_is_cxx11_and_links(compat_bin):
    assert os.access(compat_bin, os.X_OK)
    r = subprocess.run([compat_bin, "nosuchmode", "-config", "/nonexistent"], capture_output=True, text=True)
    assert r.returncode == 3 and "conf can not open" in r.stderr  # errors surface as codes, no abort


def _run(compat_bin, *args):
    r = subprocess.run([compat_bin] + list(args), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.gpu
def test_compat_ps_client(compat_bin, gpu, tmp_path):
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    out = _run(compat_bin, "ps", "-config", str(conf))
    assert "ps ok" in out and "routed=0" in out


def _free_port():
    from conftest import free_port
    return free_port()


@pytest.mark.gpu
def test_compat_ps_client_routed_rccl_world1(compat_bin, gpu, tmp_path):
    """The multi-rank code path (owner routing, RCCL exchange) at world 1."""
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    env = dict(os.environ, SWPS_ROUTE="1", MASTER_ADDR="127.0.0.1", SWPS_BOOTSTRAP_PORT=str(_free_port()))
    r = subprocess.run([compat_bin, "ps", "-config", str(conf)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "routed=1" in r.stdout


@pytest.mark.gpu
def test_compat_ps_client_two_ranks(compat_bin, gpu, tmp_path):
    """Two C++ ranks on one GPU over the library's TCP transport: keys shared
    by both ranks get both pushes as separate AdaGrad steps in rank order;
    the last rank pulls again after rank 0 finished (rank 0 keeps serving)."""
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF + "[server]\nfrag_num: 1000\n")
    port = str(_free_port())
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   SWPS_BOOTSTRAP_PORT=port, SWPS_TRANSPORT="tcp", HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([compat_bin, "ps", "-config", str(conf)], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, o + e
        assert "routed=1" in o and "world=2" in o


@pytest.mark.gpu
@pytest.mark.parametrize("ipc", ["0", "1"])
def test_compat_w2v_main_two_ranks_matches_python_driver(compat_bin, lib, gpu, tmp_path, ipc):
    """apps/word2vec/w2v.cpp's main on two C++ ranks (one GPU, TCP transport):
    each rank trains its own corpus, the library runs the key-sharded
    exchange (swps_w2v_shard_comm) — every rank's dumped shard equals the one
    the Python driver over gloo produces (tests/dist_w2v_dump.py).  ipc = 1:
    the Cluster's exchanges through the IPC path (SWPS_COMM_IPC=1)."""
    import sys
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    data = [zipf_corpus(str(tmp_path / ("c%d.txt" % r)), 70 + 25 * r, 200, seed=51 + r) for r in range(2)]
    cpp_out = str(tmp_path / "cpp_param.txt")
    port = str(_free_port())
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   SWPS_BOOTSTRAP_PORT=port, SWPS_TRANSPORT="tcp", HSA_ENABLE_IPC_MODE_LEGACY="0", SWPS_COMM_IPC=ipc)
        procs.append(subprocess.Popen([compat_bin, "w2v", "-config", str(conf), "-data", data[rank], "-niters", "2",
                                       "-output", cpp_out], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, o + e
    py_out = str(tmp_path / "py_param.txt")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "tests", "dist_w2v_dump.py"), "--data", ",".join(data), "--out", py_out],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for rank in range(2):  # w2v.cpp:54-56: the main names its rank's file, finalize writes exactly that
        a = sorted(open("%s-%d.txt" % (cpp_out, rank)).read().splitlines())
        b = sorted(open("%s.%d" % (py_out, rank)).read().splitlines())
        assert len(a) > 0 and a == b, rank


@pytest.mark.gpu
def test_compat_w2v_and_s2v_mains_match_python(compat_bin, lib, gpu, tmp_path):
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    corpus = zipf_corpus(str(tmp_path / "c.txt"), 90, 200, seed=41)
    cpp_dump = str(tmp_path / "cpp_param.txt")
    _run(compat_bin, "w2v", "-config", str(conf), "-data", corpus, "-niters", "2", "-output", cpp_dump)
    cpp_dump += "-0.txt"
    t = lib.Table("w2v", dim=16, capacity=1 << 22, dtype="f32", learning_rate=0.7)
    w = lib.Word2Vec(t, window=3, negative=4, minibatch=20, sample=1e-3, alpha=0.05)
    w.load_text(corpus)
    w.init()
    w.train(2)
    py_dump = str(tmp_path / "py_param.txt")
    t.dump(py_dump)
    assert sorted(open(cpp_dump).read().splitlines()) == sorted(open(py_dump).read().splitlines())
    # sent2vec over integer-token sentences against those word vectors' keys
    ints = int_corpus(str(tmp_path / "s.txt"), 60, 150, seed=42)
    wv = str(tmp_path / "wv.txt")
    with open(wv, "w") as f:  # integer keys for the atoi-keyed sentences
        rng = np.random.default_rng(3)
        for k in range(1, 151):
            f.write("%d\t%s\t%s\n" % (k, " ".join("%g" % x for x in rng.normal(0, .05, 16)),
                                     " ".join("%g" % x for x in rng.normal(0, .05, 16))))
    cpp_sent = str(tmp_path / "cpp_sent.txt")
    _run(compat_bin, "s2v", "-config", str(conf), "-data", ints, "-niters", "3", "-wordvec", wv, "-output", cpp_sent)
    t2 = lib.Table("w2v", dim=16, capacity=1 << 22, dtype="f32", learning_rate=0.7)
    s = lib.Sent2Vec(t2, window=3, negative=4, minibatch=20, niters=3, alpha=0.05)
    s.load_word_vector(wv)
    s.load_text(ints)
    s.train()
    py_sent = str(tmp_path / "py_sent.txt")
    s.dump(py_sent)
    assert open(cpp_sent).read() == open(py_sent).read()


@pytest.mark.gpu
def test_compat_lr_main_matches_python(compat_bin, lib, gpu, tmp_path):
    conf = tmp_path / "demo.conf"
    conf.write_text(LR_CONF)
    out = str(tmp_path / "err.txt")
    data = os.path.join(GOLDEN, "lr_data.txt")
    _run(compat_bin, "lr", "-config", str(conf), "-data", data, "-niters", "4", "-output", out)
    t = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=200)
    m.load_text(data)
    m.init()
    err = m.train(4)
    assert np.array_equal(np.loadtxt(out), err)


@pytest.mark.parametrize("case,code", [("push_body", 3), ("push_unknown", 3), ("pull_body", 3)])
def test_compat_access_method_rules_fail_loudly(compat_bin, tmp_path, case, code):
    """An access method with its own apply_push_value / init_param body and
    no declared rule, or a rule the library lacks, fails with
    SWPS_E_UNSUPPORTED before any GPU work (accessmethod.h:16-33: the library
    cannot run host bodies on the device)."""
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    r = subprocess.run([compat_bin, "rules", "-config", str(conf), "-case", case], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == code and "error -7" in r.stderr, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("case,rules", [("plain", "init_mode=1 push_rule=0"), ("push_declared", "init_mode=1 push_rule=0")])
def test_compat_access_method_rules_resolve(compat_bin, gpu, tmp_path, case, rules):
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    out = _run(compat_bin, "rules", "-config", str(conf), "-case", case)
    assert rules in out


@pytest.mark.gpu
def test_compat_lr_train_dump_then_predict_mode(compat_bin, lib, gpu, tmp_path):
    """lr.cpp's two modes: train and finalize(param path) dumps the shard;
    the predict mode (load_param, then predict) reproduces the Python
    mirror's predictions from that dump, one per line at ostream precision 6
    (lr.cpp:240-300,488-504)."""
    conf = tmp_path / "demo.conf"
    conf.write_text(LR_CONF)
    data = os.path.join(GOLDEN, "lr_data.txt")
    param = str(tmp_path / "param.txt")
    _run(compat_bin, "lr", "-config", str(conf), "-data", data, "-niters", "3", "-output", str(tmp_path / "e.txt"),
         "-param", param)
    pred = str(tmp_path / "pred.txt")
    _run(compat_bin, "lrpredict", "-config", str(conf), "-data", data, "-param", param, "-output", pred)
    t = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05)
    t.load(param)
    m = lib.LR(t, minibatch=200)
    m.load_text(data)
    m.init()
    p, _ = m.predict()
    lines = open(pred).read().splitlines()
    assert len(lines) == len(p) > 0
    assert lines == ["%g" % x for x in p]
    # the dump covers every key of the data: nothing is re-initialised, so the
    # predictions equal those of the trained model itself (to the dump's 6 digits)
    t2 = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05)
    m2 = lib.LR(t2, minibatch=200)
    m2.load_text(data)
    m2.init()
    m2.train(3)
    p2, _ = m2.predict()
    assert np.allclose(p, p2, rtol=1e-4, atol=1e-6)


# ---- the reference's own mains, UNCHANGED (tests/cpp/build_ref_apps.py) -----
LR_REF_CONF = """[ worker ]
minibatch: 200
nthreads: 1
[ server ]
initial_learning_rate: 0.05
frag_num: 1000
out_param_prefix: %s
"""


def _ref_apps():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "cpp"))
    import build_ref_apps
    return build_ref_apps


def test_host_body_rules_are_recognised(lib, tmp_path):
    """Access methods in the reference's shape with host bodies and no declared
    rule (lr.cpp:45-80's form): the bodies are run on probe values and matched
    to the device's gen_float init (SWPS_INIT_FLCG) / zero init and AdaGrad /
    SGD push rules without consuming global_random(); a body that matches no
    device rule fails with SWPS_E_UNSUPPORTED (-7)."""
    out = str(tmp_path / "probe")
    cmd = ["g++", "-std=c++11", "-O1", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "probe_rules.cpp"), "-L" + os.path.join(ROOT, "swiftmpi_amd", "lib"),
           "-lswps", "-Wl,-rpath," + os.path.join(ROOT, "swiftmpi_amd", "lib"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    conf = tmp_path / "c.conf"
    conf.write_text(LR_CONF)
    r = subprocess.run([out, str(conf)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines == ["flcg_adagrad init=2 push=0 seed_ok=1", "zero_sgd init=0 push=1 seed_ok=1",
                     "half_adagrad error -7", "flcg_momentum error -7"], lines


def test_process_rand_is_libc_rand(tmp_path):
    """swift_snails::process_rand() (the apps' Vec::randInit / WParam stream, kept apart from the
    ROCm runtime's own srand()/rand() calls) returns what glibc's rand() does after srand(1) — the
    default — call for call, over 10^6 calls; and after srand(7) for ProcessRand(7)."""
    src = tmp_path / "pr.cpp"
    src.write_text('#include <cstdio>\n#include <cstdlib>\n#include "swiftmpi_compat.h"\n'
                   "int main() {\n"
                   "  for (int i = 0; i < 1000000; i++) if (swift_snails::process_rand()() != rand()) return 1;\n"
                   "  srand(7); swift_snails::ProcessRand r(7);\n"
                   "  for (int i = 0; i < 100000; i++) if (r() != rand()) return 2;\n"
                   "  std::puts(\"ok\"); return 0;\n}\n")
    out = str(tmp_path / "pr")
    r = subprocess.run(["g++", "-std=c++11", "-O2", "-I" + os.path.join(ROOT, "include"), str(src), "-o", out],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([out], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.returncode, r.stdout)


def test_reference_mains_compile_unchanged(lib):
    """apps/word2vec/w2v.cpp, w2v_local.cpp, apps/logistic/lr.cpp and apps/sent2vec/sent2vec.cpp, read
    where they lie under /root/reference, compile with g++ -std=c++11 against
    include/swiftmpi/ (the reference's include names) and link libswps.so;
    the binaries run (usage path, no GPU work)."""
    b = _ref_apps()
    if not os.path.isdir(b.REF):
        pytest.skip("no reference tree here (the GPU box uses the binaries built in the build container)")
    bins = b.build()
    assert set(bins) == {"w2v", "w2v_local", "lr", "sent2vec"}
    r = subprocess.run([bins["lr"], "-mode"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "missing parameter" in r.stderr and "Train Mode" in r.stdout
    r = subprocess.run([bins["w2v"]], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Word2Vec application" in r.stdout
    r = subprocess.run([bins["sent2vec"]], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Doc2Vec" in r.stdout


def _ref_bin(name):
    bins = _ref_apps().binaries()
    if name not in bins:
        pytest.skip("reference mains not built (tests/cpp/build_ref_apps.py needs /root/reference)")
    return bins[name]


@pytest.mark.gpu
def test_reference_w2v_main_unchanged_equals_compat_driver(compat_bin, gpu, tmp_path):
    """w2v.cpp itself (Word2Vec<MiniBatch>, server_t, Cluster, global_mpi)
    trains on the GPU and dumps exactly what the compat driver's Word2VecApp
    does (which test_compat_w2v_and_s2v_mains_match_python ties to the Python
    mirror)."""
    ref = _ref_bin("w2v")
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    corpus = zipf_corpus(str(tmp_path / "c.txt"), 90, 200, seed=41)
    a, b = str(tmp_path / "ref_param"), str(tmp_path / "compat_param")
    _run(ref, "-config", str(conf), "-data", corpus, "-niters", "2", "-output", a)
    _run(compat_bin, "w2v", "-config", str(conf), "-data", corpus, "-niters", "2", "-output", b)
    la, lb = open(a + "-0.txt").read().splitlines(), open(b + "-0.txt").read().splitlines()
    assert len(la) > 100 and sorted(la) == sorted(lb)


@pytest.mark.gpu
def test_reference_w2v_local_main_unchanged(lib, gpu, tmp_path):
    """w2v_local.cpp (word2vec.h: atoi keys, a vocabulary and unigram table per
    minibatch) = the Python mirror's minibatch_vocab mode on the same corpus."""
    ref = _ref_bin("w2v_local")
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    corpus = int_corpus(str(tmp_path / "c.txt"), 80, 150, seed=43)
    out = str(tmp_path / "param")
    _run(ref, "-config", str(conf), "-data", corpus, "-niters", "2", "-output", out)
    t = lib.Table("w2v", dim=16, capacity=1 << 22, dtype="f32", learning_rate=0.7)
    w = lib.Word2Vec(t, window=3, negative=4, minibatch=20, sample=1e-3, alpha=0.05, key_mode="atoi",
                     minibatch_vocab=True)
    w.load_text(corpus)
    w.init()
    w.train(2)
    py = str(tmp_path / "py.txt")
    t.dump(py)
    la, lb = open(out + "-0.txt").read().splitlines(), open(py).read().splitlines()
    assert len(la) > 50 and sorted(la) == sorted(lb)


@pytest.mark.gpu
def test_reference_lr_main_unchanged_matches_oracle(lib, oracle_mod, gpu, tmp_path):
    """lr.cpp itself: its LR class learns on the host through the unchanged
    PS API (pull_with_barrier / push_with_barrier with its own BinaryBuffer
    operators) against the HBM shard; its access methods' host bodies are
    recognised as the device's gen_float init (SWPS_INIT_FLCG) and AdaGrad
    rules.  The trained dump (server.out_param_prefix + ".txt") matches the
    oracle's lr.cpp restatement, and predict mode (load_param, predict) gives
    the Python mirror's predictions from that dump."""
    ref = _ref_bin("lr")
    prefix = str(tmp_path / "lr_param")
    conf = tmp_path / "lr.conf"
    conf.write_text(LR_REF_CONF % prefix)
    data = os.path.join(GOLDEN, "lr_data.txt")
    r = subprocess.run([ref, "-mode", "train", "-config", str(conf), "-dataset", data, "-niters", "3"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    got = {}
    for line in open(prefix + ".txt"):
        k, v = line.split("\t")
        got[int(k)] = float(v)
    orc = oracle_mod.LR(data, 200, 0.05)
    orc.train(3)
    ko, wo, _ = orc.params()
    assert sorted(got) == [int(k) for k in ko]
    gw = np.array([got[int(k)] for k in ko])
    assert np.allclose(gw, wo, rtol=2e-5, atol=1e-6), np.abs(gw - wo).max()
    pred = str(tmp_path / "pred.txt")
    r = subprocess.run([ref, "-mode", "predict", "-config", str(conf), "-dataset", data, "-param_path",
                        prefix + ".txt", "-out_prefix", pred, "-niters", "1"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    p_ref = np.loadtxt(pred)
    t = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05)
    t.load(prefix + ".txt")
    m = lib.LR(t, minibatch=200)
    m.load_text(data)
    m.init()
    p, _ = m.predict()
    assert len(p_ref) == len(p) > 0 and np.allclose(p_ref, p, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_reference_lr_predict_partial_dump(lib, oracle_mod, gpu, tmp_path):
    """lr.cpp predict mode over a dump that lacks two thirds of the data's keys
    (ADVICE r04): ClusterServer::load assigns the dumped rows without drawing
    (server.h:49-62 never calls init_param), and each minibatch's pull gives the
    keys the server lacks LRPullAccessMethod::init_param's gen_float() draws in
    the key set's iteration order (lr.cpp:45-50, 240-295) — the predictions
    equal the oracle's restatement of that predict mode."""
    ref = _ref_bin("lr")
    data = os.path.join(GOLDEN, "lr_data.txt")
    t0 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    m0 = lib.LR(t0, minibatch=200)
    m0.load_text(data)
    m0.init()
    k0, _, _ = m0.params()
    keys = k0[::3]
    vals = np.array(["%g" % (0.25 + 1e-3 * i) for i in range(len(keys))], dtype=np.float32)
    dump = str(tmp_path / "partial.txt")
    with open(dump, "w") as f:
        for k, x in zip(keys, vals):
            f.write("%d\t%g\n" % (k, x))
    prefix = str(tmp_path / "lr_param")
    conf = tmp_path / "lr.conf"
    conf.write_text(LR_REF_CONF % prefix)
    pred = str(tmp_path / "pred.txt")
    r = subprocess.run([ref, "-mode", "predict", "-config", str(conf), "-dataset", data, "-param_path", dump,
                        "-out_prefix", pred, "-niters", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    p_ref = np.loadtxt(pred)
    orc = oracle_mod.LR(data, 200, 0.05)
    orc.load(keys, vals)
    p_orc = orc.predict_mode()
    assert len(p_ref) == len(p_orc) > 0
    assert np.allclose(p_ref, p_orc, rtol=2e-6, atol=1e-6), np.abs(p_ref - p_orc).max()


@pytest.mark.gpu
def test_flcg_table_load_draws_nothing(lib, gpu, tmp_path):
    """An SWPS_INIT_FLCG table (lr.cpp's gen_float init_param): load / assign
    insert the dumped keys without moving the float-LCG stream, so the first
    pulled miss gets the stream's first draw."""
    import torch
    seq = _flcg_seq(64)
    dump = str(tmp_path / "d.txt")
    with open(dump, "w") as f:
        for k in range(1, 41):
            f.write("%d\t%g\n" % (k, 0.5))
    t = lib.Table("lr", capacity=1024, dtype="f32", learning_rate=0.05, init="flcg")
    t.load(dump)
    keys = torch.arange(100, 110, dtype=torch.int64, device="cuda")
    got = t.pull(keys)[:, 0].cpu().numpy()
    assert np.array_equal(got, seq[:10]), (got, seq[:10])
    old = t.pull(torch.arange(1, 5, dtype=torch.int64, device="cuda"))[:, 0].cpu().numpy()
    assert (old == np.float32(0.5)).all()


def _flcg_seq(n):
    """gen_float() of swift_snails::Random (utils/random.h:33-36): y = y * 4903917 + 11 from
    ULONG_MAX / 2, value (float)y / 2^64 with (float)y rounded to nearest even."""
    out, y = np.zeros(n, dtype=np.float32), (2 ** 64 - 1) // 2
    for i in range(n):
        y = (y * 4903917 + 11) % 2 ** 64
        b, q = y.bit_length(), y
        if b > 24:
            sh = b - 24
            q, r = y >> sh, y & ((1 << sh) - 1)
            if r > 1 << (sh - 1) or (r == 1 << (sh - 1) and q & 1):
                q += 1
            q <<= sh
        out[i] = np.float32(q / 2.0 ** 64)
    return out


@pytest.mark.gpu
def test_reference_sent2vec_main_unchanged_matches_oracle(oracle_mod, lib, gpu, tmp_path):
    """sent2vec.cpp itself: WordMiniBatch over word2vec.h's host MiniBatch (gather_keys / pull /
    table / param / clear over the PS API on the HBM shard) and its own fp64 learn_instance on the
    host.  The dump covers 120 of the corpus's 150 keys, so pulls insert the rest with the server's
    rand() rows (the in-process server's WParam per pulled key, accessmethod.h:63-70).  Its output
    file (sentence id, "Vec:", D values at 6 digits) = the oracle's S2V (fp32 storage like the
    shard; rand() moved by Cluster::initialize's two port binds before the load) within 1e-5."""
    ref = _ref_bin("sent2vec")
    conf = tmp_path / "demo.conf"
    conf.write_text(W2V_CONF)
    corpus = int_corpus(str(tmp_path / "s.txt"), 90, 150, seed=44)
    dump = word_dump(str(tmp_path / "w.txt"), 120, 16, seed=45)
    out = str(tmp_path / "sent.txt")
    _run(ref, "-config", str(conf), "-data", corpus, "-wordvec", dump, "-niters", "2", "-output", out)
    orc = oracle_mod.S2V(corpus, 16, window=3, negative=4, minibatch=20, niters=2, table_size=10 ** 8,
                         storage_f32=True, rand_offset=2)
    orc.load_words(dump)
    orc.train()
    io, vo, _ = orc.docs()
    ids, vecs = [], []
    for line in open(out):
        sid, body = line.rstrip("\n").split("\t", 1)
        assert body.startswith("Vec:\t")
        ids.append(int(sid))
        vecs.append([float(x) for x in body[5:].split()])
    assert len(ids) == len(io) > 50 and np.array_equal(np.array(ids, dtype=np.uint64), io)
    vecs = np.array(vecs)
    assert vecs.shape == vo.shape
    assert np.allclose(vecs, vo, rtol=1e-5, atol=1e-7), np.abs(vecs - vo).max()
