"""Host sanitizers over the native engine (SURVEY.md §5 "Race detection /
sanitizers"): the standalone self-test (csrc/tools/engine_selftest.cpp —
rules invariants vs flood fill, featurizer structure, encoder, threaded
featurization and the MCTS forest) must run clean under ASan+UBSan and TSan."""
import shutil
import subprocess

import pytest

from alphago_amd import _build


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san,games", [("", 40), ("address,undefined", 24), ("thread", 8)])
def test_engine_selftest_under_sanitizer(san, games):
    exe = _build.build_selftest(san)
    r = subprocess.run([exe, str(games)], capture_output=True, text=True, timeout=600,
                       env={"TSAN_OPTIONS": "halt_on_error=1", "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
                            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
