"""Checkpoints in the TF-1.x layout:

    <dir>/checkpoint                          CheckpointState text proto (max_to_keep = 5)
    <dir>/model.ckpt-<N>.index                TensorBundle SSTable  } written by the native
    <dir>/model.ckpt-<N>.data-00000-of-00001  raw tensor bytes      } writer (csrc/ckpt)
    <dir>/model.ckpt-<N>.meta                 dtg graph manifest (JSON; TF's binary MetaGraphDef is not
                                              reproduced -- SURVEY §7.5 item 5 open decision)
    <dir>/graph.pbtxt                         GraphDef text proto of the default graph (node name, op type,
                                              inputs, ^control inputs, device, variable dtype/shape), written
                                              by CheckpointSaverHook / Supervisor like TF (dtg.graph.GraphDef)

Keys are variable op names (``Variable``, ``Variable_1``, ``global_step``, ``g/Variable``, ...),
plus the optimizer slots the parameter servers created (``g/Variable/Adagrad``).  Local variables
are not saved.  Works for graph variables and for :class:`FlatParams`-backed models
(``save_flat`` / ``restore_flat``: one key per parameter, fp32 masters).
"""
import json
import os
import re
import time

import numpy as np
import torch

from .. import graph as G

# TF DataType enum
_TF_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.int64): 9,
          np.dtype(np.uint16): 14}
_NP_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 14: np.uint16, 19: np.float16}


def _rt():
    from .. import _runtime
    return _runtime


def write_tensors(prefix, named_arrays):
    items = []
    for name, a in named_arrays:
        a = np.array(a, order="C")  # 0-d stays 0-d
        items.append((name, _TF_DT[a.dtype], list(a.shape), a.tobytes()))
    _rt().write_bundle(prefix, items)


def read_tensors(prefix, verify=True):
    out = {}
    for name, dt, shape, raw in _rt().read_bundle(prefix, verify):
        out[name] = np.frombuffer(raw, dtype=_NP_DT[dt]).reshape(shape).copy()
    return out


# ---- CheckpointState ---------------------------------------------------------------------------
class CheckpointState:
    def __init__(self, model_checkpoint_path, all_model_checkpoint_paths):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = list(all_model_checkpoint_paths)


def _state_path(d, latest_filename=None):
    return os.path.join(d, latest_filename or "checkpoint")


def update_checkpoint_state(save_dir, model_checkpoint_path, all_model_checkpoint_paths, latest_filename=None):
    def rel(p):
        return os.path.relpath(p, save_dir) if os.path.isabs(p) and os.path.dirname(p) == os.path.abspath(save_dir) \
            else (os.path.basename(p) if os.path.dirname(os.path.abspath(p)) == os.path.abspath(save_dir) else p)
    lines = ['model_checkpoint_path: "%s"' % rel(model_checkpoint_path)]
    lines += ['all_model_checkpoint_paths: "%s"' % rel(p) for p in all_model_checkpoint_paths]
    tmp = _state_path(save_dir, latest_filename) + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, _state_path(save_dir, latest_filename))


def get_checkpoint_state(checkpoint_dir, latest_filename=None):
    p = _state_path(checkpoint_dir, latest_filename)
    if not os.path.exists(p):
        return None
    model, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths)\s*:\s*"(.*)"', line)
        if not m:
            continue
        path = m.group(2)
        if not os.path.isabs(path):
            path = os.path.join(checkpoint_dir, path)
        if m.group(1) == "model_checkpoint_path":
            model = path
        else:
            allp.append(path)
    return CheckpointState(model, allp) if model else None


def checkpoint_exists(prefix):
    return os.path.exists(prefix + ".index")


def latest_checkpoint(checkpoint_dir, latest_filename=None):
    st = get_checkpoint_state(checkpoint_dir, latest_filename)
    if st and checkpoint_exists(st.model_checkpoint_path):
        return st.model_checkpoint_path
    return None


class CheckpointReader:
    """tf.train.NewCheckpointReader equivalent."""

    def __init__(self, prefix):
        self._prefix = prefix
        self._idx = _rt().read_index(prefix)
        self._vals = None

    def get_variable_to_shape_map(self):
        return {k: list(v[1]) for k, v in self._idx.items()}

    def get_variable_to_dtype_map(self):
        return {k: _NP_DT[v[0]] for k, v in self._idx.items()}

    def has_tensor(self, name):
        return name in self._idx

    def get_tensor(self, name):
        if self._vals is None:
            self._vals = read_tensors(self._prefix)
        return self._vals[name]


def load_checkpoint(ckpt_dir_or_file):
    p = latest_checkpoint(ckpt_dir_or_file) if os.path.isdir(ckpt_dir_or_file) else ckpt_dir_or_file
    return CheckpointReader(p)


# ---- Saver -----------------------------------------------------------------------------------
def _np_of(t):
    if isinstance(t, torch.Tensor):
        t = t.detach()
        if t.dtype == torch.bfloat16:
            return t.view(torch.int16).cpu().numpy().view(np.uint16)
        return t.cpu().numpy()
    return np.asarray(t)


class Saver:
    def __init__(self, var_list=None, max_to_keep=5, keep_checkpoint_every_n_hours=10000.0, include_ps_slots=True,
                 save_relative_paths=False, filename=None):
        self._var_list = var_list
        self.max_to_keep = max_to_keep
        self._include_slots = include_ps_slots
        self._last = []

    def _vars(self):
        if self._var_list is None:
            return G.get_collection(G.GraphKeys.GLOBAL_VARIABLES)
        if isinstance(self._var_list, dict):
            return list(self._var_list.values())
        return list(self._var_list)

    def _names(self):
        if isinstance(self._var_list, dict):
            return list(self._var_list.keys())
        return [v.op.name for v in self._vars()]

    def _collect(self):
        arrays = []
        seen = set()
        tasks = set()
        for name, v in zip(self._names(), self._vars()):
            arrays.append((name, _np_of(v.read_value())))
            seen.add(name)
            if getattr(v, "remote", False):
                tasks.add(v.ps_task)
        if self._include_slots:  # optimizer slots created on the PS (e.g. g/Variable/Adagrad)
            for task in sorted(tasks):
                from ..variables import client_for
                c = client_for(*task)
                names = [n for n, _, _ in c.list() if n not in seen and "/" in n and n.rsplit("/", 1)[0] in seen]
                for n, a in zip(names, c.read(names) if names else []):
                    arrays.append((n, a))
                    seen.add(n)
        for fm in self._flat_models():  # eager GPU models (register_flat_model): parameter-name keys
            for n, a in fm.arrays():
                if n in seen:
                    raise ValueError("checkpoint key %r is both a graph variable and a model parameter" % n)
                arrays.append((n, a))
                seen.add(n)
        return arrays

    def _flat_models(self):
        return G.get_collection(FLAT_MODELS) if self._var_list is None else []

    def save(self, sess, save_path, global_step=None, latest_filename=None, meta_graph_suffix="meta",
             write_meta_graph=True, write_state=True):
        if global_step is not None:
            if not isinstance(global_step, (int, np.integer)):
                global_step = int(np.asarray(sess._read(global_step) if hasattr(sess, "_read") else
                                             global_step.read_value().item()))
            prefix = "%s-%d" % (save_path, int(global_step))
        else:
            prefix = save_path
        d = os.path.dirname(os.path.abspath(prefix))
        os.makedirs(d, exist_ok=True)
        arrays = self._collect()
        write_tensors(prefix, arrays)
        if write_meta_graph:
            with open(prefix + "." + meta_graph_suffix, "w") as f:
                json.dump({"format": "dtg-graph-manifest-v1", "time": time.time(),
                           "variables": [{"name": n, "shape": list(a.shape), "dtype": str(a.dtype)} for n, a in arrays]},
                          f, indent=1)
        if write_state:
            self._last = [p for p in self._last if p != prefix] + [prefix]
            while self.max_to_keep and len(self._last) > self.max_to_keep:
                old = self._last.pop(0)
                for suf in (".index", ".data-00000-of-00001", ".meta"):
                    try:
                        os.remove(old + suf)
                    except OSError:
                        pass
            update_checkpoint_state(d, prefix, self._last, latest_filename)
        return prefix

    def restore(self, sess, save_path):
        vals = read_tensors(save_path)
        restored = []
        for fm in self._flat_models():
            fm.restore(vals, save_path)
            restored.extend(fm.names())
        by_name = dict(zip(self._names(), self._vars()))
        tasks = set()
        for name, v in by_name.items():
            if name not in vals:
                raise KeyError("Key %s not found in checkpoint %s" % (name, save_path))
            v.load(torch.from_numpy(vals[name]), create=True)
            restored.append(name)
            if getattr(v, "remote", False):
                tasks.add(v.ps_task)
        if self._include_slots and tasks:
            from ..variables import client_for
            task = sorted(tasks)[0]
            for n, a in vals.items():
                if n not in by_name and "/" in n:
                    owner = by_name.get(n.rsplit("/", 1)[0])
                    t = owner.ps_task if owner is not None and getattr(owner, "remote", False) else task
                    client_for(*t).create(n, a, True)
        return restored

    @property
    def last_checkpoints(self):
        return list(self._last)


# ---- flat-buffer models ---------------------------------------------------------------------
FLAT_MODELS = "dtg_flat_models"  # graph collection of _FlatModel saveables (Saver / CheckpointSaverHook)


class _FlatModel:
    """A FlatParams model (and its fused optimizer) as a Saver saveable: the same keys as :func:`save_flat`."""

    def __init__(self, flat, optimizer=None):
        self.flat, self.optimizer = flat, optimizer

    def arrays(self):
        return flat_arrays(self.flat, self.optimizer)

    def names(self):
        return [n for n, _ in self.flat.named_masters()]

    def restore(self, vals, what="checkpoint"):
        load_flat_arrays(self.flat, vals, self.optimizer, None, what)


def register_flat_model(flat, optimizer=None):
    """Make ``Saver()`` (and so MonitoredTrainingSession's CheckpointSaverHook and its restore) checkpoint a
    FlatParams model: one key per parameter name, its buffers, and the optimizer's slots and step.  Idempotent
    per ``flat``; a later call with an optimizer attaches it."""
    for fm in G.get_collection(FLAT_MODELS):
        if fm.flat is flat:
            if optimizer is not None:
                fm.optimizer = optimizer
            return fm
    fm = _FlatModel(flat, optimizer)
    G.add_to_collection(FLAT_MODELS, fm)
    return fm


SLOT_LAYOUT_KEY = "dtg/slot_layout"
SLOT_LAYOUT_LOGICAL = 1
def flat_arrays(flat, optimizer=None):
    """The named fp32 arrays of a FlatParams model -- one key per parameter (its module name), the module's
    buffers, and with ``optimizer`` its slots as ``<param>/<slot>`` plus ``optimizer/step`` -- as written by
    :func:`save_flat` and by :class:`Saver` for models registered with ``dtg.train.register_flat_model``."""
    arrays = [(n, _np_of(v)) for n, v in flat.named_masters()]
    for n, b in flat.module.named_buffers():
        arrays.append((n, _np_of(b)))
    if optimizer is not None:
        from ..parallel.flat import _view_like
        # slots are stored in LOGICAL parameter order (since f74dff1); only the first checkpoints held
        # channels_last conv slots in physical [K,R,S,C] order -- restore_flat(legacy_slot_layout=True)
        arrays.append((SLOT_LAYOUT_KEY, np.array(SLOT_LAYOUT_LOGICAL, dtype=np.int64)))
        arrays.append(("optimizer/step", np.array(int(getattr(optimizer, "step_count", 0)), dtype=np.int64)))
        for g in flat:
            for k, buf in g.state.items():
                for i, n in enumerate(g.names):
                    # same logical layout as the master (channels_last conv weights included), so
                    # '<param>/<slot>' is element-aligned with '<param>' for any reader
                    arrays.append(("%s/%s" % (n, k), _np_of(_view_like(buf, g.offsets[i], g.params[i]))))
    return arrays


def save_flat(flat, prefix, global_step=None, extra=None, max_to_keep=5, state_dir=None, optimizer=None):
    """Checkpoint a FlatParams model (+ module buffers, optimizer state) as a TensorBundle."""
    arrays = flat_arrays(flat, optimizer)
    if global_step is not None:
        arrays.append(("global_step", np.array(int(global_step), dtype=np.int64)))
        prefix = "%s-%d" % (prefix, int(global_step))
    for k, v in (extra or {}).items():
        arrays.append((k, np.asarray(v)))
    write_tensors(prefix, arrays)
    d = state_dir or os.path.dirname(os.path.abspath(prefix))
    st = get_checkpoint_state(d)
    allp = [p for p in (st.all_model_checkpoint_paths if st else []) if p != prefix] + [prefix]
    while max_to_keep and len(allp) > max_to_keep:
        old = allp.pop(0)
        for suf in (".index", ".data-00000-of-00001", ".meta"):
            try:
                os.remove(old + suf)
            except OSError:
                pass
    update_checkpoint_state(d, prefix, allp)
    return prefix


def restore_flat(flat, prefix, optimizer=None, legacy_slot_layout=None):
    """Restore what :func:`save_flat` wrote.  With ``optimizer``: its slots too (created when the optimizer
    has not stepped yet) and its step count.  Returns the checkpoint's global step (or None).

    Slots are read in logical parameter order, which every save_flat since f74dff1 writes -- with or without
    the ``dtg/slot_layout`` marker (added later).  Only checkpoints from before f74dff1 hold channels_last
    conv slots in physical [K,R,S,C] order; converting those is opt-in (``legacy_slot_layout=True`` or
    ``DTG_LEGACY_SLOT_LAYOUT=1``), and refused for a checkpoint that carries the logical marker."""
    vals = read_tensors(prefix)
    load_flat_arrays(flat, vals, optimizer, legacy_slot_layout, prefix)
    return int(vals["global_step"]) if "global_step" in vals else None


def load_flat_arrays(flat, vals, optimizer=None, legacy_slot_layout=None, what="checkpoint"):
    """Load the arrays :func:`flat_arrays` produced (a dict name -> ndarray) into ``flat`` (and ``optimizer``)."""
    from ..parallel.flat import _view_like
    if legacy_slot_layout is None:
        legacy_slot_layout = os.environ.get("DTG_LEGACY_SLOT_LAYOUT") == "1"
    marked = int(vals.get(SLOT_LAYOUT_KEY, -1)) == SLOT_LAYOUT_LOGICAL
    if legacy_slot_layout and marked:
        raise ValueError("%s: legacy_slot_layout requested, but the checkpoint is marked logical" % what)
    logical = not legacy_slot_layout
    with torch.no_grad():
        for g in flat:
            if optimizer is not None:  # slots present in the checkpoint but not yet allocated
                for n in g.names:
                    for key in vals:
                        if key.startswith(n + "/") and "/" not in key[len(n) + 1:] and key[len(n) + 1:] not in g.state:
                            k = key[len(n) + 1:]
                            # the optimizer initialises what the checkpoint does not hold (alignment padding)
                            optimizer.new_slot(g, k) if hasattr(optimizer, "new_slot") else g.state_buffer(k)
            for i, n in enumerate(g.names):
                if n not in vals:
                    raise KeyError("Key %s not found in %s" % (n, what))
                mv = g.master_view(i)
                mv.copy_(torch.from_numpy(vals[n]).view(mv.shape))
                for k, buf in g.state.items():
                    key = "%s/%s" % (n, k)
                    if key in vals:
                        p = g.params[i]
                        sv = _view_like(buf, g.offsets[i], p)
                        src = torch.from_numpy(vals[key])
                        if not logical and p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(
                                memory_format=torch.channels_last):
                            o, c, r, s_ = p.shape  # legacy physical [K,R,S,C] slot order
                            src = src.reshape(o, r, s_, c).permute(0, 3, 1, 2)
                        sv.copy_(src.reshape(sv.shape))
            g.refresh_mirror()
        for n, b in flat.module.named_buffers():
            if n in vals:
                b.copy_(torch.from_numpy(vals[n]).view(b.shape))
    if optimizer is not None and "optimizer/step" in vals and hasattr(optimizer, "step_count"):
        optimizer.step_count = int(vals["optimizer/step"])
        if hasattr(optimizer, "hyper"):
            optimizer.hyper[1].fill_(float(optimizer.step_count))
