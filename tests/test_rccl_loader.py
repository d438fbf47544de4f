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
