"""dtg.ops -- hand-written gfx950 HIP kernels exposed as differentiable PyTorch ops.

GPU bf16 tensors run on dtg's own kernels (csrc/kernels/*.hip); CPU tensors run the PyTorch
reference of the same op so the distributed plumbing can be tested without a GPU.
"""
from ._native import lib, available  # noqa: F401
from .batchnorm import batch_norm_act  # noqa: F401
from .loss import softmax_cross_entropy  # noqa: F401
from .gemm import gemm, linear  # noqa: F401
from .conv import conv2d  # noqa: F401
from . import transformer  # noqa: F401
from .pool import max_pool2d, global_avg_pool  # noqa: F401
from . import optim_kernels  # noqa: F401
