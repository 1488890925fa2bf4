"""HipMCL expansion step on MI355X: prune / select / recover and the phased expansion SpGEMM.

Mirrors (gabe-raulet/CombBLAS):
    MCLPruneRecoverySelect(A, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion)
                                                    include/CombBLAS/ParFriends.h:185-353
    MemEfficientSpGEMM<SR>(A, B, phases, hardThreshold, selectNum, recoverNum, recoverPct,
                           kselectVersion, computationKernel, perProcessMemory)
                                                    include/CombBLAS/ParFriends.h:449-730
on local (1-rank) matrices.  The distributed versions live in combblas_amd.dist.  Every call goes
through libcbgpu (cbg_mcl_prune, cbg_col_range, cbg_col_concat, cbg_spgemm_local); there is no CPU
path.  MCL's defaults (Applications/MCL.cpp:147-151): prunelimit 1e-4, select 1100, recover_num
1400, recover_pct 0.9, kselectVersion 1.
"""
import ctypes

from . import _abi
from ._abi import CbgError

MCL_DEFAULTS = dict(hardThreshold=1.0 / 10000.0, selectNum=1100, recoverNum=1400, recoverPct=0.9)


def _prune_result(ctx, res, hardThreshold, selectNum, recoverNum, recoverPct):
    out = _abi.CscResult()
    st = _abi.MclStats()
    _abi.check(ctx._lib.cbg_mcl_prune(ctx._ptr, ctypes.byref(res), float(hardThreshold), int(selectNum),
                                      int(recoverNum), float(recoverPct), ctypes.byref(out), ctypes.byref(st)),
               "cbg_mcl_prune")
    return out, {"recovered": st.recovered, "selected": st.selected,
                 "recovered_after_select": st.recovered_after_select, "nnz_in": st.nnz_in, "nnz_out": st.nnz_out}


def MCLPruneRecoverySelect(A, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1):
    """Prune A (a local SpDCCols / SpTuples holding complete columns) in place, as ParFriends.h:185-353.
    kselectVersion only picks the reference's CPU selection algorithm (Kselect1 vs Kselect2, same
    k-th value), so it does not change the result.  Returns the branch statistics."""
    out, stats = _prune_result(A._ctx, A._res, hardThreshold, selectNum, recoverNum, recoverPct)
    A._ctx._lib.cbg_result_free(A._ctx._ptr, ctypes.byref(A._res))
    A._res = out
    return stats


def _col_range(ctx, res, c0, c1):
    out = _abi.CscResult()
    _abi.check(ctx._lib.cbg_col_range(ctx._ptr, ctypes.byref(res), int(c0), int(c1), ctypes.byref(out)),
               "cbg_col_range")
    return out


def _col_concat(ctx, parts):
    arr = (_abi.CscResult * len(parts))(*parts)
    out = _abi.CscResult()
    _abi.check(ctx._lib.cbg_col_concat(ctx._ptr, arr, len(parts), ctypes.byref(out)), "cbg_col_concat")
    return out


def phase_ranges(ncol, phases):
    """ColSplit pieces (SpDCCols.cpp:927-1086): ncol // phases columns each, the last takes the rest."""
    step = ncol // phases
    return [(p * step, ncol if p == phases - 1 else (p + 1) * step) for p in range(phases)]


def MemEfficientSpGEMM(SR, A, B, phases, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1,
                       computationKernel=1, perProcessMemory=0, stats=None):
    """C = prune(A * B) computed in `phases` column phases of B (ParFriends.h:449-730), 1 rank.

    Each phase multiplies A by a column piece of B, prunes the piece (MCLPruneRecoverySelect) and
    keeps only the pruned piece; the pieces are concatenated.  computationKernel (1 hash, 2 heap)
    picks the reference's CPU kernel; the device kernel is the same for both.  perProcessMemory > 0
    raises `phases` the way the reference does for a 1-process grid (input, output and k-select
    memory against the budget in GB, ParFriends.h:479-521)."""
    from . import SpTuples, _as_tuples   # local import: package __init__ imports this module lazily
    ctx = A._ctx
    if A.getncol() != B.getnrow():
        raise CbgError(_abi.EDIM, "MemEfficientSpGEMM")
    if phases < 1 or phases >= A.getncol():
        phases = 1
    if perProcessMemory > 0:
        phases = _phases_for_memory(SR, A, B, selectNum, recoverNum, perProcessMemory, phases)
    pieces, totals = [], {"recovered": 0, "selected": 0, "recovered_after_select": 0, "multiplies": 0,
                          "nnz_unpruned": 0, "phases": phases}
    try:
        for (c0, c1) in phase_ranges(B.getncol(), phases):
            if phases == 1:
                Bp = B
            else:
                Bp = type(B)._from_result(ctx, _col_range(ctx, B._res, c0, c1))
            Cp = ctx.spgemm(A, Bp, SR, sort=True)
            if Bp is not B:
                Bp.free()
            totals["multiplies"] += Cp.multiplies
            totals["nnz_unpruned"] += Cp.getnnz()
            res, st = _prune_result(ctx, Cp._res, hardThreshold, selectNum, recoverNum, recoverPct)
            Cp.free()
            pieces.append(res)
            for k in ("recovered", "selected", "recovered_after_select"):
                totals[k] += st[k]
        if len(pieces) == 1:
            out = pieces.pop()
        else:
            out = _col_concat(ctx, pieces)
    finally:
        for r in pieces:
            ctx._lib.cbg_result_free(ctx._ptr, ctypes.byref(r))
    out.multiplies = totals["multiplies"]
    if stats is not None:
        stats.update(totals)
    return SpTuples._from_result(ctx, out)


def _phases_for_memory(SR, A, B, selectNum, recoverNum, perProcessMemory, phases):
    """ParFriends.h:479-521 with p = 1: asquareNNZ from the symbolic pass (EstPerProcessNnzSUMMA)."""
    from . import EstimateLocalFLOP   # noqa: F401  (symbolic pass via cbg_estimate)
    ctx = A._ctx
    m, z = ctypes.c_int64(0), ctypes.c_int64(0)
    va, vb = A._view(), B._view()
    _abi.check(ctx._lib.cbg_estimate(ctx._ptr, ctypes.byref(va), ctypes.byref(vb), ctypes.byref(m),
                                     ctypes.byref(z)), "cbg_estimate")
    per_in, per_out = 8 * 2 + 8, 8 * 2 + 8
    input_mem = A.getnnz() * per_in * 4
    asq_mem = int(z.value) * per_out * 2
    ncolB = max(1, B.getncol())
    d = -(-int(z.value) // ncolB)
    k = min(max(selectNum, recoverNum), d)
    ksel_mem = ncolB * k * 8 * 3
    out_mem = ncolB * k * per_in * 2
    remaining = perProcessMemory * 1000000000 - input_mem - out_mem
    if remaining > 0:
        phases = 1 + (asq_mem + ksel_mem) // remaining
    return max(1, min(int(phases), max(1, A.getncol() - 1)))
