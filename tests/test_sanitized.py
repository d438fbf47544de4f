"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU oracle.

The sanitized executable (bin_asan/svm_serial, built by ``python -m svm355.build --sanitize``) runs
the whole serial pipeline — CSV parse (including malformed rows), scaling, SMO, prediction, model
dump — and must exit cleanly with no sanitizer report."""
import subprocess

import numpy as np
import pytest

from svm355 import build


@pytest.fixture(scope="module")
def asan_exe():
    return build.build_sanitized()


def _run(exe, args, tmp_path):
    env = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=23", "UBSAN_OPTIONS": "print_stacktrace=1",
           "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=600, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_asan_serial_synthetic(asan_exe, tmp_path):
    out = _run(asan_exe, ["--synthetic", "400,100", "--threads", "4", "--model-dir", "m", "--json", "s.json"], tmp_path)
    assert "Final SV count" in out and (tmp_path / "m" / "final_b.txt").exists()


def test_asan_serial_csv_with_malformed_rows(asan_exe, tmp_path):
    rng = np.random.default_rng(0)
    X = rng.integers(0, 256, size=(300, 20))
    lab = rng.integers(0, 10, size=300)
    lines = ["," .join([f"f{i}" for i in range(20)] + ["label"])]
    for i in range(300):
        lines.append(",".join(str(v) for v in X[i]) + f",{lab[i]}")
        if i % 50 == 7:
            lines.append("")       # blank line
            lines.append("5")      # fewer than 2 fields: skipped like the reference
    (tmp_path / "d_train_data.csv").write_text("\n".join(lines) + "\n")
    (tmp_path / "d_test_data.csv").write_text("\n".join(lines[:120]) + "\n")
    out = _run(asan_exe, ["--dataset", "d", "--gamma", "0.01"], tmp_path)
    assert out.startswith("n = 300")


# ---- the threaded host code: apps/svm_threads.cpp runs the strict-loopback
# cascades (star P = 2/3/8, tree P = 2/4/8), the same cascades over HostCommTransport (its callbacks
# served by loopback ranks in threads), an abort mid-round, a checkpoint + resume, the decomposition
# oracle's 8-thread worker team and its distributed form on 8 loopback / 4 hostcomm thread ranks with a
# rank failing mid-solve.  Every scenario checks its own result (bit-identical models, the failing
# rank's error on every rank); the sanitizers check the memory and the synchronisation.

@pytest.fixture(scope="module")
def thread_exes():
    return build.build_sanitized_threads()


def _run_threads(exe, args, env_extra, timeout):
    env = {"PATH": "/usr/bin:/bin", "TMPDIR": "/tmp", **env_extra}
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "ALL SCENARIOS OK" in r.stdout, out[-5000:]
    for bad in ("runtime error", "AddressSanitizer", "LeakSanitizer", "ThreadSanitizer"):
        assert bad not in out, out[-5000:]
    return r.stdout


def test_asan_ubsan_threaded_cascades_hostcomm_and_decomp(thread_exes):
    out = _run_threads(thread_exes[0], [], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=23",
                                            "UBSAN_OPTIONS": "print_stacktrace=1"}, timeout=900)
    for line in ("cascade hostcomm star P=8", "cascade loopback tree P=8", "cascade checkpoint + resume",
                 "decomp distributed, 8 loopback thread ranks", "decomp rank failing mid-solve"):
        assert line in out


def test_tsan_threaded_cascades_hostcomm_and_decomp(thread_exes):
    """TSan (ROCm clang's runtime: gcc 11's libtsan misreads libstdc++'s condition-variable waits), the
    full scenario list (~1.5 min)."""
    out = _run_threads(thread_exes[1], [], {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"}, timeout=900)
    assert "cascade hostcomm tree P=8" in out and "decomp distributed, 4 hostcomm ranks" in out
