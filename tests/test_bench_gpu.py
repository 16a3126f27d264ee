"""bench.py as the driver runs it, on the one-GPU box: `--gpus 2` starts two
rank processes itself (no external launcher), they share cuda:0 over the
library's TCP transport (RCCL refuses two ranks on one device), and rank 0
prints one line with n_gpus 2 and the world-2 exchange block."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_gpus2_spawns_two_ranks(lib, gpu):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--tokens", "1000000", "--vocab", "50000", "--minibatch", "200", "--no-cpu-baseline", "--no-parity-leg",
           "--b100-steps", "0", "--config1-steps", "0", "--no-app-legs"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    print({k: out[k] for k in ("value", "n_gpus", "ms_per_step", "transport")}, out["exchange"])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["transport"] == "tcp" and out["transport_ranks"] == 2
    x = out["exchange"]
    assert x is not None and "world 2" in x["note"] and x["bytes_remote_per_step"] > 0 and x["a2a_per_step"] >= 2
    assert "key-sharded PS over 2 GPU(s)" in out["config"]["parallelism"]
