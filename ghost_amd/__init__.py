"""ghost_amd — MI355X-native (gfx950) implementation of GHOST's per-frame face-swap forward path.

Public surface mirrors the reference: ``ghost_amd.network.AEI_Net`` (network/AEI_Net.py) and
``ghost_amd.inference.faceshifter_batch`` (utils/inference/faceshifter_run.py).  The compute
runs in ``libghost_amd.so`` (hand-written HIP kernels, C ABI in include/ghost_amd.h).
"""
__version__ = "0.1.0"
