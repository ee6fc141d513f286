"""SURVEY §5 (race detection / sanitizers): the multithreaded native behaviours
parser (csrc/host/behaviors.cpp: row chunks parsed in parallel, private id
tables merged in chunk order) built with AddressSanitizer + UBSan and with
ThreadSanitizer, driven by tests/sanitize/behaviors_driver.cpp, which checks
that 2/5/16 threads over 1-byte chunks give exactly the sequential parse
(ids first seen late, shared ids, None histories, labelled and unlabelled
rows, a malformed late row) with no sanitizer report.  Host code only: GPU
sanitizers are not available on the pool."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

SRC = [REPO / "tests" / "sanitize" / "behaviors_driver.cpp", REPO / "news_recommendation_project_v2_amd" / "csrc" /
       "host" / "behaviors.cpp"]
BUILDS = {
    "asan_ubsan": (["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
                    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}),
    "tsan": (["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}),
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("build", sorted(BUILDS))
def test_behaviors_parser_under_sanitizer(build, tmp_path):
    flags, env = BUILDS[build]
    exe = tmp_path / f"behaviors_{build}"
    cc = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", *flags, *map(str, SRC), "-o", str(exe)],
                        capture_output=True, text=True, timeout=300)
    assert cc.returncode == 0, cc.stderr[-3000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env={**os.environ, **env})
    report = run.stderr
    assert run.returncode == 0, report[-4000:]
    for marker in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "LeakSanitizer"):
        assert marker not in report, report[-4000:]
    assert "0 failures" in run.stdout
