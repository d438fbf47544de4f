"""svm355 — an MI355X-native kernel-SVM trainer (SMO + Cascade SVM) on PyTorch-ROCm, hand-written
CDNA4 HIP kernels and RCCL over xGMI.

Capabilities of guaijiacc/Parallelizing-Support-Vector-Machine-Training-with-GPU-and-MPI,
re-designed for gfx950:

* ``svm355.models.SVC``              RBF SVM, first-order SMO (reference semantics), CPU oracle or GPU
* ``svm355.models.OneVsRestSVC``     all digits one-vs-rest over ONE resident Gram (10 SMO solves)
* ``svm355.parallel.CascadeSVM``     classical tree and modified two-layer star Cascade SVM: one native
                                     driver over RCCL (a thread per GPU, or one rank per process under
                                     torchrun) or the loopback transport (CPU oracle / one-GPU rehearsal)
* ``svm355.parallel.DistributedSVC`` ONE SMO over the GPUs of a node: points and Gram slabs split over
                                     GPUs, per-iteration candidates exchanged over xGMI; the single-GPU
                                     trajectory bit for bit (``--parallel smo``)
* ``svm355.utils.data``              CSV I/O, one-vs-rest labels, min-max scaling, synthetic MNIST
* ``svm355.ops``                     device kernels (exact-integer int8-MFMA and f64-MFMA RBF Grams,
                                     persistent SMO solvers, HBM row cache, predict)
* CLIs: ``python -m svm355 {serial,gpu,sweep,cascade}`` and native ``bin/svm_serial``, ``bin/svm_gpu``
"""
import os as _os

# RCCL between processes needs dmabuf IPC (the legacy mode fails on these hosts); effective only if
# set before the first HIP call of the process.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from .utils.config import SVMParams  # noqa: E402
from .utils.data import Dataset, MinMaxScaler, load_csv, one_vs_rest, synthetic_mnist, write_csv
from .models.multiclass import OneVsRestSVC
from .models.svc import SVC

__all__ = ["SVMParams", "Dataset", "MinMaxScaler", "load_csv", "one_vs_rest", "synthetic_mnist", "write_csv",
           "SVC", "OneVsRestSVC", "CascadeSVM", "DistributedSVC"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "CascadeSVM":
        from .parallel.cascade import CascadeSVM

        return CascadeSVM
    if name == "DistributedSVC":
        from .parallel.dsmo import DistributedSVC

        return DistributedSVC
    raise AttributeError(name)
