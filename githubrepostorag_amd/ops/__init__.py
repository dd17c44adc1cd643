"""MI355X (gfx950) op library.

Every op dispatches on the tensor's device: device tensors run the
hand-written HIP kernels from ``csrc/kernels`` (``libgrag_kernels.so``), CPU
tensors run an fp32 PyTorch reference of the same op (used by the CPU test
tier and as the numerics oracle for the GPU tests).
"""
from . import attention, elementwise, linear, norm, sampling, topk  # noqa: F401
from ._lib import available, lib, lib_path, loaded_path  # noqa: F401
