"""librbx's RCCL merge inside a process that already runs torch.distributed over RCCL (bench.py's
C4 leg at N > 1): one rank, every call of the path on the GPU (tools/rccl_check.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_rccl_merge_in_torch_process():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_check.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"counts_unchanged": true' in r.stdout
