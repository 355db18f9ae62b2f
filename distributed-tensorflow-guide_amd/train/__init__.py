"""dtg.train -- the tf.train surface the reference scripts use."""
from ..cluster import ClusterSpec, Server  # noqa: F401
from ..placement import replica_device_setter  # noqa: F401
from .optimizer import (Optimizer, GradientDescentOptimizer, AdagradOptimizer, MomentumOptimizer,  # noqa: F401
                        AdamOptimizer, get_global_step, create_global_step, get_or_create_global_step)
from .sync_replicas import SyncReplicasOptimizer  # noqa: F401
from .hooks import (SessionRunHook, SessionRunArgs, SessionRunContext, SessionRunValues, StopAtStepHook,  # noqa: F401
                    NanTensorHook, NanLossDuringTrainingError, LoggingTensorHook, StepCounterHook,
                    CheckpointSaverHook, SummarySaverHook, GlobalStepWaiterHook, FinalOpsHook, FeedFnHook,
                    ProfilerHook)
from .session import (MonitoredTrainingSession, MonitoredSession, Supervisor, Scaffold, SessionManager,  # noqa: F401
                      Coordinator, ChiefSessionCreator, WorkerSessionCreator, Session)
from .saver import (Saver, latest_checkpoint, get_checkpoint_state, update_checkpoint_state,  # noqa: F401
                    checkpoint_exists, CheckpointReader, load_checkpoint, save_flat, restore_flat,
                    register_flat_model, flat_arrays)
from .eager import broadcast_training_state  # noqa: F401
from . import eager  # noqa: F401
from .summary import FileWriter  # noqa: F401

NewCheckpointReader = CheckpointReader


def barrier(name, count=None, timeout=600.0, ps_task=0):
    """Rendezvous of ``count`` tasks (default: all workers) on PS task ``ps_task``.

    Replaces the reference's bootstrap sleeps (chief ``sleep(10)`` after pushing its initial
    values, DOWNPOUR/DOWNPOUR.py:129-131; ``sleep(40)`` in SSGD-diff-LR/ssgd.py:95) with a real
    barrier in the native PS service."""
    from ..variables import _this_server, client_for
    s = _this_server()
    if s is None:
        return True
    n = count if count is not None else s.cluster.num_tasks("worker")
    return client_for("ps", ps_task).barrier(name, int(n), float(timeout))
from ..graph import write_graph  # noqa: F401,E402  (tf.train.write_graph)
