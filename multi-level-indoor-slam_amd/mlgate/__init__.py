"""mlgate -- MI355X-native semantic loop-closure gate.

Drop-in for the hot path of wadewilliamsw1234/Multi-level-Indoor-SLAM's
``scripts.semantic_gating`` (VPR descriptors, all-keyframes cosine kNN, floor gate,
geometric verification), computed by hand-written gfx950 HIP kernels behind the C ABI
in include/mlgate.h.
"""
__version__ = "0.1.0"
