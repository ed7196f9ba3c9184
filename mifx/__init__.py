"""mifx — an MI355X-native ML pipeline framework (TFX-style components, KFP-compatible DSL,
PyTorch-ROCm models with hand-written gfx950 HIP kernels, RCCL data parallelism)."""
__version__ = "0.1.0"
