"""Two ranks (gloo, sharing cuda:0) drive the real libswps sharded path on
OVERLAPPING vocabularies / feature spaces and match the lockstep multi-rank
oracle (each rank's push its own AdaGrad step, in rank order; server.h:
156-176).  Runs tests/dist_shared_check.py under torch.distributed.run as a
child process (its ranks are fresh processes; this one only waits)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from conftest import free_port
    return free_port()


@pytest.mark.parametrize("modes", ["f64,parity", "fast,lr", "fast300", "bfp300", "fp32str,bfp32str"])
def test_shared_keys_two_ranks_match_lockstep_oracle(lib, oracle_mod, gpu, modes):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_shared_check.py"), "--backend", "gloo", "--modes", modes]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-3000:])
    print(r.stderr[-3000:])
    assert r.returncode == 0 and "SHARED OK" in r.stdout
