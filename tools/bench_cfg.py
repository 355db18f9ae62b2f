#!/usr/bin/env python3
"""bench.py with a forced native configuration, for in-step A/B runs (tools/ab_bench.sh takes environments,
so the choice is passed as DTG_AB_BN_CFG / DTG_AB_GEMM_CFG and applied here before bench.py runs):

    DTG_AB_BN_CFG=-1 python tools/bench_cfg.py [bench.py flags]     # BN-epilogue GEMMs without the expand kernel
    DTG_AB_SET=models.resnet_fused._DXW=0 python tools/bench_cfg.py  # a module switch (dtg.<module>.<name>=<int>)
    DTG_AB_STAGES=0:2,1:3 python tools/bench_cfg.py   # conv LDS schedules per pass (0 fwd, 1 dgrad, 2 wgrad, 3 stem)
    DTG_AB_STEM_STREAM=0 python tools/bench_cfg.py    # the tiled stem conv instead of the streaming one
    DTG_AB_HALO=0 python tools/bench_cfg.py           # the implicit-GEMM stage-1 3x3 forward instead of the halo one
    DTG_AB_HALO_DGRAD=0 python tools/bench_cfg.py     # the implicit-GEMM stage-1 3x3 dgrad instead of the halo one
    DTG_AB_HALO_WGRAD=0 python tools/bench_cfg.py     # the implicit-GEMM stage-1 3x3 wgrad instead of the halo one
    DTG_AB_LIN_WGRAD=0 python tools/bench_cfg.py      # the implicit-GEMM stage-2..4 3x3 wgrads instead of the linear halo
    DTG_AB_LIN_WGRAD=256 python tools/bench_cfg.py    # the linear-halo wgrads on 256 workgroups (halo: DTG_AB_HALO_WGRAD=128)
    DTG_AB_EXPAND256=0 python tools/bench_cfg.py      # stage-3 conv3 (K = 256) on the tiled BN GEMM, not the expand kernel
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import dtg  # noqa: E402,F401
from dtg.ops._native import lib  # noqa: E402

if os.environ.get("DTG_AB_HALO"):  # 0: the implicit-GEMM forward for the stage-1 3x3 (conv_halo.hip EPI 0)
    lib().conv_halo_fwd_set(int(os.environ["DTG_AB_HALO"]))
if os.environ.get("DTG_AB_STEM_STREAM"):  # 0: the tiled stem conv instead of the streaming one
    lib().stem_stream_set(int(os.environ["DTG_AB_STEM_STREAM"]))
if os.environ.get("DTG_AB_HALO_DGRAD"):  # 0: the implicit-GEMM dgrad for the stage-1 3x3 (conv_halo.hip EPI 1)
    lib().conv_halo_dgrad_set(int(os.environ["DTG_AB_HALO_DGRAD"]))
if os.environ.get("DTG_AB_HALO_WGRAD"):  # 0: the implicit-GEMM wgrad for the stage-1 3x3 (conv_halo.hip)
    lib().conv_halo_wgrad_set(int(os.environ["DTG_AB_HALO_WGRAD"]))
if os.environ.get("DTG_AB_LIN_WGRAD"):  # 0: the implicit-GEMM wgrad for the stage-2..4 3x3s (conv_halo.hip lin)
    lib().conv_lin_wgrad_set(int(os.environ["DTG_AB_LIN_WGRAD"]))
if os.environ.get("DTG_AB_EXPAND256"):  # 0: the tiled BN-statistics GEMM for K = 256 (stage-3 conv3) instead of expand
    lib().gemm_expand_k256_set(int(os.environ["DTG_AB_EXPAND256"]))
if os.environ.get("DTG_AB_EXPAND_S2"):  # 0: the implicit-GEMM conv for the stage-2 1x1 / s2 projection forward
    lib().gemm_expand_s2_set(int(os.environ["DTG_AB_EXPAND_S2"]))
if os.environ.get("DTG_AB_POOL_ROWS"):  # 0: the row-parallel stem max-pool forward instead of the row-walking one
    lib().stem_pool_rows_set(int(os.environ["DTG_AB_POOL_ROWS"]))
if os.environ.get("DTG_AB_BN_CFG"):
    lib().gemm_bn_force_cfg(int(os.environ["DTG_AB_BN_CFG"]))
for item in filter(None, os.environ.get("DTG_AB_STAGES", "").split(",")):  # "<pass>:<schedule>", conv_set_stages
    which, sched = item.split(":")
    lib().conv_set_stages(int(which), int(sched))
for item in filter(None, os.environ.get("DTG_AB_SET", "").split(",")):
    path, val = item.split("=")
    mod, name = path.rsplit(".", 1)
    import importlib
    setattr(importlib.import_module("dtg." + mod), name, type(getattr(importlib.import_module("dtg." + mod), name))(int(val)))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
