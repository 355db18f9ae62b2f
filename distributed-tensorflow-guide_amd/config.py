"""ConfigProto / GPUOptions (Multiple-GPUs-Single-Machine/dist_mult_gpu_sing_mach.py:45-49).

``log_device_placement`` prints the variable -> task placement when a session is created;
``gpu_options.visible_device_list`` selects the HIP device of a worker (a PyTorch-ROCm caching
allocator replaces TF's BFC allocator, so ``allow_growth`` / ``allocator_type`` are accepted and
have no further effect).
"""


class GPUOptions:
    def __init__(self, allow_growth=False, allocator_type="BFC", visible_device_list="",
                 per_process_gpu_memory_fraction=0.0):
        self.allow_growth = allow_growth
        self.allocator_type = allocator_type
        self.visible_device_list = visible_device_list
        self.per_process_gpu_memory_fraction = per_process_gpu_memory_fraction


class ConfigProto:
    def __init__(self, log_device_placement=False, allow_soft_placement=False, gpu_options=None,
                 device_filters=None, inter_op_parallelism_threads=0, intra_op_parallelism_threads=0):
        self.log_device_placement = log_device_placement
        self.allow_soft_placement = allow_soft_placement
        self.gpu_options = gpu_options or GPUOptions()
        self.device_filters = device_filters or []
        self.inter_op_parallelism_threads = inter_op_parallelism_threads
        self.intra_op_parallelism_threads = intra_op_parallelism_threads

    def hip_device(self):
        """The torch device a worker should use under this config."""
        import torch
        if not torch.cuda.is_available():
            return torch.device("cpu")
        vis = self.gpu_options.visible_device_list
        idx = int(str(vis).split(",")[0]) if str(vis).strip() else 0
        return torch.device("cuda", idx % torch.cuda.device_count())
