"""C callers of the drop-in boundary: tests/c/stats_replay.c includes
include/dmx.h and links -ldmx exactly as a C user of the reference's deflate_ext.h would
 and automates tests/check_lld.c's replay contract (:20-39, :56-79);
tests/c/host_asan.c runs the library's host C under AddressSanitizer + UBSan."""
import glob
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "build", "c")
GOLD = os.path.join(REPO, "tests", "golden")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "c")])
    return OUT


def test_host_c_asan_ubsan(built):
    """Every truncation and bit flip of the reference's PNG IDAT streams through our inflate,
    Adler-32 combine, the generators and the boundary's error paths: no sanitizer finding
    (leak detection on; the ROCm runtime's own allocations suppressed, tests/c/lsan.supp),
    every corrupt stream rejected with -E_*.  On a GPU box deflate_compress really encodes."""
    env = dict(os.environ, LSAN_OPTIONS="suppressions=" + os.path.join(REPO, "tests", "c", "lsan.supp"))
    p = subprocess.run([os.path.join(built, "host_asan")] + sorted(glob.glob(os.path.join(GOLD, "idat", "*.zlib"))),
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "0 failed checks" in p.stdout


def test_stats_replay_links(built):
    """The C caller resolves every symbol it uses from libdmx.so (no GPU needed to link/load)."""
    p = subprocess.run(["ldd", os.path.join(built, "stats_replay")], capture_output=True, text=True)
    assert "libdmx.so" in p.stdout and "not found" not in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("stats", ["ref", "exact"])
@pytest.mark.parametrize("case", ["bee", "text", "mixed", "sw4096"])
def test_stats_replay_on_gpu(built, tmp_path, case, stats):
    import deflate_compression_amd as D
    text = D.gen_text(150000, 5).tobytes()
    data = {"bee": open(os.path.join(GOLD, "bee_movie_script.txt"), "rb").read(), "text": text,
            "mixed": text[:40000] + bytes(50000) + D.gen_random(30000, 3).tobytes() + text[:70000],
            "sw4096": text[:90000]}[case]
    fi = tmp_path / "in"
    fi.write_bytes(data)
    args = [os.path.join(built, "stats_replay"), str(fi)] + (["4096"] if case == "sw4096" else [])
    p = subprocess.run(args, capture_output=True, text=True, timeout=120, env=dict(os.environ, DMX_STATS=stats))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "stats_replay ok" in p.stdout
