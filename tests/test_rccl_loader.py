"""The RCCL the device library runs on (csrc/hip/rccl_api.h): the library of its own headers."""
def test_rccl_runtime_is_the_headers_library_even_inside_pytorch():
    """The device library loads the librccl its headers belong to (rccl_api.h, dlopen with RTLD_LOCAL |
    RTLD_DEEPBIND), not the copy PyTorch bundles (RCCL 2.26.6 against 2.27.7 headers before round 4):
    no skew, on a CPU host too (ncclGetVersion needs no device)."""
    import torch  # noqa: F401  (loads torch's own librccl first, as in every bench process)

    from svm355.parallel.rccl import rccl_info

    info = rccl_info()
    assert info["rccl_skew"] is False and info["rccl_header"] == info["rccl_runtime"] != "unknown"
    assert info["rccl_path"].endswith("librccl.so.1") and "torch" not in info["rccl_path"]


def test_unloadable_rccl_is_an_error_not_an_abort():
    """SVM355_RCCL_LIB pointing nowhere: the entry points that need RCCL report an error through the C ABI
    (svmd_nccl_unique_id) instead of letting a C++ exception terminate the process -- the per-process
    bench then falls back to the gloo transport (tests/test_gpu_bench.py)."""
    import subprocess
    import sys
    from pathlib import Path

    code = ("from svm355.parallel.rccl import RcclRank\n"
            "from svm355._native import NativeError\n"
            "try:\n    RcclRank.unique_id()\nexcept NativeError as e:\n    print('ERR', e)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=Path(__file__).resolve().parents[1],
                       env={**__import__("os").environ, "SVM355_RCCL_LIB": "/nonexistent/librccl.so"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ERR" in r.stdout and "cannot load /nonexistent/librccl.so" in r.stdout
