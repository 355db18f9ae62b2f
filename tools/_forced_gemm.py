"""forced_gemm(cfg, ...): the production GEMM (cfg 0, dtg._C heuristic) or one forced tile configuration from the
lab extension (cfg != 0: dtg._lab.gemm_cfg -- the forced table, 99 = 256x256 8-phase, 96-98 = its persistent
form), with the production binding's positional arguments (A, a_kc, B, b_kc, out, alpha, beta, bias, act,
split_k, aux, aux_mode)."""
from dtg.ops._native import lab, lib


def forced_gemm(cfg, A, a_kc, B, b_kc, out, alpha=1.0, beta=0.0, bias=None, act=0, split_k=0, aux=None, aux_mode=0):
    if cfg == 0:
        return lib().gemm(A, a_kc, B, b_kc, out, alpha, beta, bias, act, split_k, aux, aux_mode)
    if not lab().gemm_cfg(cfg, A, a_kc, B, b_kc, out, alpha, beta, bias, act, max(1, split_k), aux, aux_mode):
        raise ValueError("forced GEMM configuration %d does not apply to this problem" % cfg)
