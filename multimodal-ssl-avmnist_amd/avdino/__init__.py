"""avdino -- MI355X-native multimodal-DINO training path for AVMNIST.

Host side (Python, PyTorch-ROCm for memory/streams/distributed) over libavdino.so, the
hand-written HIP kernels for gfx950 (include/avdino.h).  Mirrors the reference's
(wardvdnb/Multimodal-SSL-AVMNIST) model classes and CLI for the run_dino.py hot path.
"""
__version__ = "0.1.0"
