"""dtg -- an MI355X-native distributed-training framework with the capabilities and example-script
API of the Distributed-TensorFlow-Guide (ClusterSpec/Server, parameter-server algorithms, sync
replicas, sessions, hooks, TF-layout checkpoints), re-designed for gfx950: PyTorch-ROCm, hand-written
HIP/CDNA4 kernels (csrc/kernels) and RCCL over xGMI.
"""
__version__ = "0.1.0"
