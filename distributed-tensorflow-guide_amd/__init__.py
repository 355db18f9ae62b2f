"""dtg -- an MI355X-native distributed-training framework with the capabilities and example-script
API of the Distributed-TensorFlow-Guide (ClusterSpec/Server, parameter-server algorithms, sync
replicas, sessions, hooks, TF-layout checkpoints), re-designed for gfx950: PyTorch-ROCm,
hand-written HIP/CDNA4 kernels (csrc/kernels) and RCCL over xGMI.

Layers:
  L0  native: csrc/kernels (HIP), csrc/ps (PS service), csrc/ckpt (TensorBundle)  -> dtg._C, dtg._runtime
  L1  dtg.ClusterSpec / dtg.Server                                               (cluster.py)
  L2  dtg.device / dtg.train.replica_device_setter / collections                 (placement.py, graph.py)
  L3  models (toy graph ops, MNIST, ResNet-50, BERT-base)                         (graph.py, models/)
  L4  optimizers, SyncReplicasOptimizer, PS algorithms, all-reduce DP             (train/, parallel/)
  L5  MonitoredTrainingSession / Supervisor / Scaffold / hooks / Saver            (train/)
  L6/7 examples/ with the reference's directory names, run.sh and flags
"""
__version__ = "0.1.0"

from .graph import (GraphKeys, Graph, Tensor, Op, get_default_graph, reset_default_graph,  # noqa: F401
                    add_to_collection, get_collection, get_collection_ref, control_dependencies, name_scope,
                    device, constant, placeholder, no_op, group, identity, convert_to_tensor, square, abs, sqrt, exp, log,
                    relu, tanh, reduce_mean, reduce_sum, reduce_max, matmul)
from .variables import (Variable, get_variable, assign, assign_add, global_variables, local_variables,  # noqa: F401
                        trainable_variables, all_variables, variables_initializer, global_variables_initializer,
                        local_variables_initializer, report_uninitialized_variables, is_variable_initialized,
                        truncated_normal, glorot_uniform_initializer, zeros_initializer, constant_initializer)
from .cluster import ClusterSpec, Server  # noqa: F401
from .placement import DeviceSpec, replica_device_setter  # noqa: F401
from .config import ConfigProto, GPUOptions  # noqa: F401
from . import train  # noqa: F401
from . import flags  # noqa: F401

import torch as _torch  # noqa: E402

float32, float64, int32, int64, bfloat16 = _torch.float32, _torch.float64, _torch.int32, _torch.int64, _torch.bfloat16
