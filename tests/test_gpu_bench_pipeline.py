"""bench.py's pipelined N > 1 timed loop at N = 1: the double-buffered
encode / gather with the comm stream, events and dmx_encode_result_async that the first
multi-GPU run takes, through RCCL on a single-rank process group.  Run as a
child process exactly as the driver would; the line must report a bit-exact round trip."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pipeline_loop_at_n1():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--pipeline-test", "1", "--steps", "3",
                        "--warmup", "1", "--cpu-budget", "0", "--real-text", "0", "--tradeoff", "",
                        "--exhaustive-steps", "0", "--long-run", "0"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["inflate_ok"] is True
    assert line["gpu_inflate"]["bit_exact"] is True
    assert "pipelined" in line["config"]["parallelism"]
    assert line["value"] > 0 and line["n_gpus"] == 1
