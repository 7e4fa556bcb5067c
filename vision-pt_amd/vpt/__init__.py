"""vpt — MI355X-native (gfx950) JiT rectified-flow training step for p1atdev/vision-pt.

Everything on the compute path runs in libvpt_hip.so (hand-written HIP/CDNA4 kernels behind the
C ABI in include/vpt_hip.h); importing this package loads it and fails loudly if it is missing.
"""

from . import _lib  # noqa: F401  (raises ImportError when libvpt_hip.so is absent)

__all__ = ["ops", "engine", "jit_train", "optim", "ddp", "config", "params", "rope"]
