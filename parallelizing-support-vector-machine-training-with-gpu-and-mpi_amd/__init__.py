"""svm355 — an MI355X-native kernel-SVM trainer (SMO + Cascade SVM) on PyTorch-ROCm, hand-written
CDNA4 HIP kernels and RCCL over xGMI.

Capabilities of guaijiacc/Parallelizing-Support-Vector-Machine-Training-with-GPU-and-MPI,
re-designed for gfx950:

* ``svm355.SVC``                     RBF SVM with the reference's semantics (stop test, clip / update
                                     arithmetic): on the GPU the SMO-type working-set decomposition
                                     solver by default (``solver="smo"``: the reference's pairwise
                                     trajectory, bit for bit the CPU oracle's); on the CPU the oracle
* ``svm355.OneVsRestSVC``            all classes one-vs-rest: the decomposition solver per class on the
                                     shared device rows (default), or one resident Gram with every
                                     pairwise class solve in one launch (``solver="batched"``)
* ``svm355.CascadeSVM``              classical tree and modified two-layer star Cascade SVM: one native
                                     driver over RCCL (a thread per GPU, or one rank per process under
                                     torchrun), over gloo (host-staged process ranks), or the loopback
                                     transport (CPU oracle / one-GPU rehearsal)
* ``svm355.DistributedDecompSVC``    the decomposition solver over the GPUs of a node (the N-GPU bench
                                     headline): selection blocks and f split over GPUs, one candidate
                                     all-gather per outer iteration; one GPU's model bit for bit
* ``svm355.DistributedSVC``          ONE pairwise SMO over the GPUs of a node, the single-GPU pairwise
                                     trajectory bit for bit (``bench.py --parallel smo``)
* ``svm355.utils.data``              CSV I/O, one-vs-rest labels, min-max scaling, synthetic MNIST
* ``svm355.ops``                     device kernels (exact-integer int8-MFMA and FP64-MFMA RBF kernel
                                     values, decomposition and persistent SMO solvers, HBM column and row
                                     caches, predict) and the CPU oracles
* CLIs: ``python -m svm355 {serial,gpu,sweep,cascade,scale,multiclass}`` and native ``bin/svm_serial``,
  ``bin/svm_gpu``, ``bin/svm_cascade``
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
           "SVC", "OneVsRestSVC", "CascadeSVM", "DistributedSVC", "DistributedDecompSVC"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "CascadeSVM":
        from .parallel.cascade import CascadeSVM

        return CascadeSVM
    if name == "DistributedDecompSVC":
        from .parallel.decomp import DistributedDecompSVC

        return DistributedDecompSVC
    if name == "DistributedSVC":
        from .parallel.dsmo import DistributedSVC

        return DistributedSVC
    raise AttributeError(name)
