"""Host AddressSanitizer / UBSan run of the engine's host-side format layer
(roaringbitmap_amd/csrc/format.cpp).

tests/asan/format_fuzz.cpp feeds the reference's own data files (the golden bitmaps and
the crashproneinput*.bin adversarial inputs, RBT/TestAdversarialInputs.java:32-55), every
truncation of them, seeded byte mutations and random value sets through parse /
from_values / runOptimize / toArray; a heap overflow, use-after-free or undefined
behaviour aborts the run.  Sanitizers run on host code only (no GPU here)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "testdata")


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("asan") / "format_fuzz")
    cmd = [gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "asan", "format_fuzz.cpp"),
           os.path.join(ROOT, "roaringbitmap_amd", "csrc", "format.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def test_format_layer_under_asan(fuzz_bin):
    files = sorted(glob.glob(os.path.join(GOLD, "*.bin")))
    assert files
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin] + files, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout

