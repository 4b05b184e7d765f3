"""bench.py's multi-rank plumbing on CPU: `--gpus N` without a launcher
starts N ranks itself, a world that differs from --gpus fails, and rank 0's stitched-stream
check (verify_stitched) accepts exactly the right stream.  The chunks here are shard streams
from the CPU oracle in the framing the HIP path emits."""
import json
import os
import subprocess
import sys
import zlib

import pytest

import deflate_compression_amd as D
from deflate_compression_amd import shard as S
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=180)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n and line["ranks_ok"]


def test_world_mismatch_exits_nonzero():
    p = _run(["--gpus", "2", "--launch-check"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "launcher started 1 rank" in p.stderr


def _shards(data: bytes, world: int, **kw):
    chunks, adlers, lens = [], [], []
    for r in range(world):
        lo, hi = S.shard_range(len(data), r, world)
        piece = data[lo:hi]
        chunks.append(O.compress(piece, flags=S.shard_flags(r, world), **kw))
        adlers.append(zlib.adler32(piece))
        lens.append(hi - lo)
    return chunks, adlers, lens


@pytest.mark.parametrize("world", [1, 2, 8])
def test_verify_stitched(world):
    data = D.gen_text(8 * 32768 + 777, 11).tobytes()
    chunks, adlers, lens = _shards(data, world, max_chain=6, lazy=True, store_check=True)
    bounds = [S.shard_range(len(data), r, world) for r in range(world)]
    pieces = [(lambda lo=lo, hi=hi: data[lo:hi]) for lo, hi in bounds]
    assert bench.verify_stitched(chunks, adlers, lens, pieces)
    # the one-stream framing: stitched == what zlib inflates to the input
    assert zlib.decompress(b"".join(chunks) + S.trailer(S.combine_adler(adlers, lens))) == data
    bad = bytearray(chunks[-1])
    bad[len(bad) // 2] ^= 0x10
    assert not bench.verify_stitched(chunks[:-1] + [bytes(bad)], adlers, lens, pieces)
    assert not bench.verify_stitched(chunks, [adlers[0] ^ 1] + adlers[1:], lens, pieces)
    if world > 1:   # a missing or a swapped chunk fails
        assert not bench.verify_stitched(chunks[1:], adlers, lens, pieces)
        assert not bench.verify_stitched(chunks[::-1], adlers, lens, pieces)
