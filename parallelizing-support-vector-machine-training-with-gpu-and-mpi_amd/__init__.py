"""svm355 — an MI355X-native kernel-SVM trainer (SMO + Cascade SVM) on PyTorch-ROCm, hand-written
CDNA4 HIP kernels and RCCL over xGMI.

Capabilities of guaijiacc/Parallelizing-Support-Vector-Machine-Training-with-GPU-and-MPI,
re-designed for gfx950:

* ``svm355.models.SVC``              RBF SVM, first-order SMO (reference semantics), CPU oracle or GPU
* ``svm355.models.OneVsRestSVC``     all digits one-vs-rest over ONE resident Gram (10 SMO solves)
* ``svm355.parallel.CascadeSVM``     classical tree and modified two-layer star Cascade SVM over
                                     ``torch.distributed`` (RCCL on GPUs, gloo on CPUs) or threads
* ``svm355.utils.data``              CSV I/O, one-vs-rest labels, min-max scaling, synthetic MNIST
* ``svm355.ops``                     device kernels (MFMA f64 RBF Gram, fused WSS, SMO step, predict)
* CLIs: ``python -m svm355 {serial,gpu,sweep,cascade}`` and native ``bin/svm_serial``, ``bin/svm_gpu``
"""
from .utils.config import SVMParams
from .utils.data import Dataset, MinMaxScaler, load_csv, one_vs_rest, synthetic_mnist, write_csv
from .models.multiclass import OneVsRestSVC
from .models.svc import SVC

__all__ = ["SVMParams", "Dataset", "MinMaxScaler", "load_csv", "one_vs_rest", "synthetic_mnist", "write_csv",
           "SVC", "OneVsRestSVC", "CascadeSVM"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "CascadeSVM":
        from .parallel.cascade import CascadeSVM

        return CascadeSVM
    raise AttributeError(name)
