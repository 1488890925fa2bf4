"""Distributed SpGEMM: CombBLAS's 2D SUMMA and 3D split SUMMA over torch.distributed.

One process per GPU.  Collectives go through torch.distributed: backend "nccl" (= RCCL over xGMI on
MI355X) in production, "gloo" in the CPU tests.  Local blocks are CSC torch tensors on the backend's
device (int64 colptr, int32 rows, values); the local multiply and the multiway merge are the
backend's (libcbgpu on the GPU: `GpuBackend`).

Reference interfaces mirrored (file:line under gabe-raulet/CombBLAS):

  CommGrid / CommGrid3D        src/CommGrid.cpp:37-76, include/CombBLAS/CommGrid3D.h:21-80
  SpParMat (2D blocks)         include/CombBLAS/SpParMat.h:451-464 (PSpGEMM), SpParMat.cpp
  SpParMat3D (col/row split)   include/CombBLAS/SpParMat3D.cpp:187-279
  Mult_AnXBn_Synch / PSpGEMM   include/CombBLAS/ParFriends.h:1004-1108, SpParMat.h:451-464
  Mult_AnXBn_SUMMA3D           include/CombBLAS/ParFriends.h:2918-3208
  3DSpGEMM multiply            3DSpGEMM/Multiplier.h:10-61 (SUMMALayer.h:24-97, Reductions.h:36-155)
  BCastMatrix / GetSetSizes    src/SpParHelper.cpp:583-627, 798-809

Layout (one formulation covers every mandated grid): the inner dimension's block k
(of the q x q layer grid) is cut into L contiguous layer parts.  Rank (l, i, j) holds
  A-side ("colsplit"): A[row block i, layer-l part of column block j]
  B-side ("rowsplit"): B[layer-l part of row block i, column block j]
Layer l runs q SUMMA stages (stage k: broadcast A(l,i,k) along grid row i and B(l,k,j) along grid
column j, multiply, keep the partial) and merges its q partials; the L layers' partials of C(i, j)
are then exchanged along the fiber (all-to-all of the layer column parts, Reductions.h:36-130) and
merged, so rank (l, i, j) ends with C[row block i, layer-l part of column block j] (colsplit, like A).
  2 GPUs: L=2, q=1 (1x1x2: no broadcast, one fiber exchange)
  4 GPUs: L=1, q=2 (2x2 SUMMA, 2 stages, no fiber exchange)
  8 GPUs: L=2, q=2 (2x2x2)
Stage k+1's broadcasts are issued (async) before stage k's multiply, so they overlap it.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import _abi

_TORCH_DT = {np.dtype(np.float64): torch.float64, np.dtype(np.float32): torch.float32,
             np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.uint8): torch.uint8}
_ABI_DT = {torch.float64: _abi.F64, torch.float32: _abi.F32, torch.int64: _abi.I64, torch.int32: _abi.I32,
           torch.uint8: _abi.BOOL}


def block_range(n, parts, idx):
    """Contiguous block `idx` of `parts` over [0, n): n // parts each, the last takes the remainder
    (CombBLAS's block distribution, e.g. SpParMat::getlocalrows / CalculateColSplitDistributionOfLayer)."""
    step = n // parts
    lo = idx * step
    hi = n if idx == parts - 1 else lo + step
    return lo, hi


def piece_range(n, q, L, blk, layer):
    """Layer `layer` part of block `blk` (q blocks, each cut into L layer parts)."""
    b0, b1 = block_range(n, q, blk)
    p0, p1 = block_range(b1 - b0, L, layer)
    return b0 + p0, b0 + p1


@dataclass
class Block:
    """Local CSC block (the SpDCCols of a SpParMat) as tensors on the backend device."""
    nrow: int
    ncol: int
    cp: torch.Tensor      # int64 [ncol + 1]
    ir: torch.Tensor      # int32 [nnz]
    val: torch.Tensor     # [nnz]

    @property
    def nnz(self):
        return int(self.ir.numel())


def block_from_host(nrow, ncol, cp, ir, val, device):
    return Block(int(nrow), int(ncol), torch.as_tensor(np.ascontiguousarray(cp, np.int64)).to(device),
                 torch.as_tensor(np.ascontiguousarray(ir, np.int32)).to(device),
                 torch.as_tensor(np.ascontiguousarray(val)).to(device))


def slice_csc(cp, ir, val, r0, r1, c0, c1):
    """Host CSC submatrix [r0, r1) x [c0, c1), rows rebased (rows stay sorted within a column)."""
    lo, hi = int(cp[c0]), int(cp[c1])
    rows = ir[lo:hi]
    keep = (rows >= r0) & (rows < r1)
    cols = np.repeat(np.arange(c1 - c0, dtype=np.int64), np.diff(cp[c0:c1 + 1]))
    cnt = np.bincount(cols[keep], minlength=c1 - c0)
    ncp = np.zeros(c1 - c0 + 1, np.int64)
    np.cumsum(cnt, out=ncp[1:])
    return ncp, (rows[keep] - r0).astype(np.int32), val[lo:hi][keep]


# ------------------------------------------------------------------------------------------- grid
class CommGrid3D:
    """layers x rows x cols process grid (CommGrid3D.h:21-80); rank = l*rows*cols + i*cols + j.
    Every rank creates every subgroup in the same order (torch.distributed.new_group contract)."""

    def __init__(self, layers, rows, cols):
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        if layers * rows * cols != self.world:
            raise ValueError(f"grid {layers}x{rows}x{cols} != world size {self.world}")
        if rows != cols:
            raise ValueError("SUMMA needs a square layer grid (CommGrid.cpp:44-50)")
        self.L, self.q = layers, rows
        self.layer, rem = divmod(self.rank, rows * cols)
        self.row, self.col = divmod(rem, cols)
        self.row_group = self.col_group = self.fiber_group = None
        for l in range(layers):
            for i in range(rows):
                g = dist.new_group([self.rank_of(l, i, j) for j in range(cols)])
                if (l, i) == (self.layer, self.row):
                    self.row_group = g
        for l in range(layers):
            for j in range(cols):
                g = dist.new_group([self.rank_of(l, i, j) for i in range(rows)])
                if (l, j) == (self.layer, self.col):
                    self.col_group = g
        for i in range(rows):
            for j in range(cols):
                g = dist.new_group([self.rank_of(l, i, j) for l in range(layers)])
                if (i, j) == (self.row, self.col):
                    self.fiber_group = g

    def rank_of(self, l, i, j):
        return l * self.q * self.q + i * self.q + j


def CommGrid(rows, cols):
    """2D grid (CommGrid.cpp:37-76) = one layer."""
    return CommGrid3D(1, rows, cols)


def grid_for(world):
    """The mandated layout per GPU count: 1 -> 1x1x1, 2 -> 1x1x2, 4 -> 2x2, 8 -> 2x2x2."""
    return {1: (1, 1, 1), 2: (2, 1, 1), 4: (1, 2, 2), 8: (2, 2, 2)}[world]


# ---------------------------------------------------------------------------------------- matrix
class SpParMat3D:
    """Local piece of a distributed matrix (SpParMat3D.cpp:187-279).  colsplit=True: A-side / output
    layout; colsplit=False: B-side (row split of the inner dimension)."""

    def __init__(self, grid, nrow, ncol, block, colsplit, backend):
        self.grid, self.nrow, self.ncol, self.block = grid, int(nrow), int(ncol), block
        self.colsplit, self.backend = colsplit, backend

    def local_range(self):
        g = self.grid
        if self.colsplit:
            return block_range(self.nrow, g.q, g.row), piece_range(self.ncol, g.q, g.L, g.col, g.layer)
        return piece_range(self.nrow, g.q, g.L, g.row, g.layer), block_range(self.ncol, g.q, g.col)

    @classmethod
    def from_global_csc(cls, grid, nrow, ncol, cp, ir, val, colsplit, backend):
        self = cls(grid, nrow, ncol, None, colsplit, backend)
        (r0, r1), (c0, c1) = self.local_range()
        lcp, lir, lval = slice_csc(cp, ir, val, r0, r1, c0, c1)
        self.block = block_from_host(r1 - r0, c1 - c0, lcp, lir, lval, backend.device)
        return self

    def getnnz(self):
        t = torch.tensor([self.block.nnz], dtype=torch.int64, device=self.backend.comm_device)
        dist.all_reduce(t)
        return int(t.item())


# ------------------------------------------------------------------------------------ collectives
def _to_comm(t, backend):
    return t if t.device == backend.comm_device else t.to(backend.comm_device)


def _from_comm(t, backend):
    return t if t.device == backend.device else t.to(backend.device)


class _BlockBcast:
    """Broadcast of one Block from `root` (global rank) within `group` (SpParHelper::BCastMatrix,
    SpParHelper.cpp:583-627).  Shapes and nnz are known to every receiver in advance (GetSetSizes)."""

    def __init__(self, blk, nrow, ncol, nnz, root, group, backend, me):
        self.backend = backend
        cd = backend.comm_device
        if me == root:
            self.cp, self.ir, self.val = _to_comm(blk.cp, backend), _to_comm(blk.ir, backend), _to_comm(blk.val, backend)
        else:
            self.cp = torch.empty(ncol + 1, dtype=torch.int64, device=cd)
            self.ir = torch.empty(nnz, dtype=torch.int32, device=cd)
            self.val = torch.empty(nnz, dtype=backend.val_dtype, device=cd)
        self.nrow, self.ncol = nrow, ncol
        self.works = [dist.broadcast(t, src=root, group=group, async_op=True) for t in (self.cp, self.ir, self.val)
                      if t.numel() > 0]

    def wait(self):
        for w in self.works:
            w.wait()
        return Block(self.nrow, self.ncol, _from_comm(self.cp, self.backend), _from_comm(self.ir, self.backend),
                     _from_comm(self.val, self.backend))


def _allgather_nnz(blk, group, size, backend):
    t = torch.tensor([blk.nnz], dtype=torch.int64, device=backend.comm_device)
    out = [torch.zeros(1, dtype=torch.int64, device=backend.comm_device) for _ in range(size)]
    dist.all_gather(out, t, group=group)
    return [int(x.item()) for x in out]


def _fiber_exchange(C, grid, backend, sr):
    """Reduce the L layers' partials of C(i, j) (Reductions.h:36-130 / ParFriends.h SUMMA3D fiber
    all-to-all): layer part m of the local partial's columns goes to the fiber's rank m, and each
    rank merges the L pieces it receives (MultiwayMergeHash semantics: SR::add in layer order).
    Layer part m of the local columns = block_range(ncol_local, L, m), which is piece_range of the
    global column block (CalculateColSplitDistributionOfLayer, SpParMat3D.cpp:576-606)."""
    L = grid.L
    bounds = [block_range(C.ncol, L, m) for m in range(L)]
    cp_host = C.cp.cpu().numpy()
    col_cnt = torch.diff(C.cp)
    nnz_split = [int(cp_host[c1] - cp_host[c0]) for (c0, c1) in bounds]
    col_split = [c1 - c0 for (c0, c1) in bounds]
    cd = backend.comm_device
    send_n = torch.tensor(nnz_split, dtype=torch.int64, device=cd)
    recv_n = torch.empty(L, dtype=torch.int64, device=cd)
    dist.all_to_all_single(recv_n, send_n, group=grid.fiber_group)
    recv_nnz = [int(x) for x in recv_n.cpu().tolist()]
    my_cols = col_split[grid.layer]
    r_cnt = torch.empty(L * my_cols, dtype=torch.int64, device=cd)
    r_ir = torch.empty(sum(recv_nnz), dtype=torch.int32, device=cd)
    r_val = torch.empty(sum(recv_nnz), dtype=backend.val_dtype, device=cd)
    dist.all_to_all_single(r_cnt, _to_comm(col_cnt, backend), [my_cols] * L, col_split, group=grid.fiber_group)
    dist.all_to_all_single(r_ir, _to_comm(C.ir, backend), recv_nnz, nnz_split, group=grid.fiber_group)
    dist.all_to_all_single(r_val, _to_comm(C.val, backend), recv_nnz, nnz_split, group=grid.fiber_group)
    r_cnt, r_ir, r_val = _from_comm(r_cnt, backend), _from_comm(r_ir, backend), _from_comm(r_val, backend)
    pieces, off = [], 0
    for m in range(L):
        cnt = r_cnt[m * my_cols:(m + 1) * my_cols]
        cp = torch.zeros(my_cols + 1, dtype=torch.int64, device=backend.device)
        torch.cumsum(cnt, 0, out=cp[1:])
        pieces.append(Block(C.nrow, my_cols, cp, r_ir[off:off + recv_nnz[m]], r_val[off:off + recv_nnz[m]]))
        off += recv_nnz[m]
    return pieces[0] if L == 1 else backend.merge(pieces, sr)


# ----------------------------------------------------------------------------------- multiplies
def Mult_AnXBn_SUMMA3D(SR, A, B, stats=None):
    """C = A * B over the semiring on the 3D grid (ParFriends.h:2918-3208).  A must be colsplit,
    B rowsplit, on the same grid; C comes back colsplit.  Dimension checks as CheckSpGEMMCompliance
    (ParFriends.h:160-181): a mismatch raises (the reference aborts with DIMMISMATCH 3002)."""
    g = A.grid
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, "Mult_AnXBn_SUMMA3D")
    if not A.colsplit or B.colsplit or B.grid is not g:
        raise ValueError("A must be colsplit and B rowsplit on the same CommGrid3D")
    be = A.backend
    q, L = g.q, g.L
    a_nnz = _allgather_nnz(A.block, g.row_group, q, be)   # pieces (l, i, k), k = 0..q-1
    b_nnz = _allgather_nnz(B.block, g.col_group, q, be)   # pieces (l, k, j)
    r0, r1 = block_range(A.nrow, q, g.row)
    ncl = B.block.ncol   # local columns of B (= of C): block `col` of B, or a phase piece of it

    def issue(k):
        k0, k1 = piece_range(A.ncol, q, L, k, g.layer)
        a = _BlockBcast(A.block, r1 - r0, k1 - k0, a_nnz[k], g.rank_of(g.layer, g.row, k), g.row_group, be, g.rank)
        b = _BlockBcast(B.block, k1 - k0, ncl, b_nnz[k], g.rank_of(g.layer, k, g.col), g.col_group, be, g.rank)
        return a, b

    partials = []
    pending = issue(0) if q > 1 else None
    for k in range(q):
        if q > 1:
            a, b = pending
            Ak, Bk = a.wait(), b.wait()
            if k + 1 < q:
                pending = issue(k + 1)   # double buffering: stage k+1 travels while stage k multiplies
        else:
            Ak, Bk = A.block, B.block
        partials.append(be.multiply(Ak, Bk, SR, stats))
    C = partials[0] if q == 1 else be.merge(partials, SR)
    if L > 1:
        C = _fiber_exchange(C, g, be, SR)
    return SpParMat3D(g, A.nrow, B.ncol, C, True, be)


def Mult_AnXBn_Synch(SR, A, B, stats=None):
    """2D SUMMA (ParFriends.h:1004-1108) = the one-layer case of the 3D driver."""
    if A.grid.L != 1:
        raise ValueError("Mult_AnXBn_Synch needs a 2D (one-layer) grid")
    return Mult_AnXBn_SUMMA3D(SR, A, B, stats)


def PSpGEMM(SR, A, B, stats=None):
    """SpParMat.h:451-464: the default distributed SpGEMM (Mult_AnXBn_Synch)."""
    return Mult_AnXBn_Synch(SR, A, B, stats)


def multiply(SR, A, B, stats=None):
    """3DSpGEMM driver entry (Multiplier.h:10-61): split-3D product on the grid A and B live on."""
    return Mult_AnXBn_SUMMA3D(SR, A, B, stats)


# ------------------------------------------------------------------------------ HipMCL expansion
def _col_slice(b, c0, c1):
    """Columns [c0, c1) of a Block (one ColSplit piece, SpDCCols.cpp:927-1086)."""
    e0, e1 = int(b.cp[c0]), int(b.cp[c1])
    return Block(b.nrow, c1 - c0, b.cp[c0:c1 + 1] - b.cp[c0], b.ir[e0:e1], b.val[e0:e1])


def _col_concat(blocks, device):
    """ColConcatenate (SpDCCols.cpp:1087-1185) of Blocks with equal nrow."""
    cps, off = [torch.zeros(1, dtype=torch.int64, device=device)], 0
    for b in blocks:
        cps.append(b.cp[1:] + off)
        off += b.nnz
    return Block(blocks[0].nrow, sum(b.ncol for b in blocks), torch.cat(cps),
                 torch.cat([b.ir for b in blocks]), torch.cat([b.val for b in blocks]))


def _gather_columns(blk, grid, nrow_global, be):
    """Complete columns for the prune: the q ranks of a processor column (col_group) each hold one
    row block of the same local columns.  Column group m = block_range(ncol, q, m) goes to column
    rank m, which stacks the q row blocks (rows offset to global).  Plays the role of the
    processor-column reductions/gathers inside Reduce(Column) and Kselect1 (SpParMat.cpp:1413-1700)."""
    q, dev, cd = grid.q, be.device, be.comm_device
    ncl = blk.ncol
    groups = [block_range(ncl, q, m) for m in range(q)]
    cp_h = blk.cp.cpu().numpy()
    nnz_split = [int(cp_h[g1] - cp_h[g0]) for (g0, g1) in groups]
    col_split = [g1 - g0 for (g0, g1) in groups]
    send_n = torch.tensor(nnz_split, dtype=torch.int64, device=cd)
    recv_n = torch.empty(q, dtype=torch.int64, device=cd)
    dist.all_to_all_single(recv_n, send_n, group=grid.col_group)
    recv_nnz = [int(x) for x in recv_n.cpu().tolist()]
    g0, g1 = groups[grid.row]
    ng = g1 - g0
    r_cnt = torch.empty(q * ng, dtype=torch.int64, device=cd)
    r_ir = torch.empty(sum(recv_nnz), dtype=torch.int32, device=cd)
    r_val = torch.empty(sum(recv_nnz), dtype=be.val_dtype, device=cd)
    dist.all_to_all_single(r_cnt, _to_comm(torch.diff(blk.cp), be), [ng] * q, col_split, group=grid.col_group)
    dist.all_to_all_single(r_ir, _to_comm(blk.ir, be), recv_nnz, nnz_split, group=grid.col_group)
    dist.all_to_all_single(r_val, _to_comm(blk.val, be), recv_nnz, nnz_split, group=grid.col_group)
    cnt = _from_comm(r_cnt, be).view(q, ng)
    r_ir, r_val = _from_comm(r_ir, be), _from_comm(r_val, be)
    cp = torch.zeros(ng + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt.sum(0), 0, out=cp[1:])
    before = torch.cumsum(cnt, 0) - cnt             # entries of column c from sources < i
    out_ir = torch.empty_like(r_ir)
    out_val = torch.empty_like(r_val)
    off = 0
    cols = torch.arange(ng, device=dev)
    for i in range(q):
        n_i = recv_nnz[i]
        if n_i:
            col = torch.repeat_interleave(cols, cnt[i])
            scp = torch.zeros(ng + 1, dtype=torch.int64, device=dev)
            torch.cumsum(cnt[i], 0, out=scp[1:])
            local = torch.arange(n_i, device=dev) - scp[col]
            dst = cp[col] + before[i, col] + local
            r0, _ = block_range(nrow_global, q, i)
            out_ir[dst] = r_ir[off:off + n_i] + r0
            out_val[dst] = r_val[off:off + n_i]
        off += n_i
    return Block(nrow_global, ng, cp, out_ir, out_val), groups


def _scatter_columns(P, grid, groups, nrow_local, be):
    """Inverse of _gather_columns: row block i of the pruned complete columns goes back to column
    rank i; each rank concatenates the q column groups of its row block."""
    q, dev, cd = grid.q, be.device, be.comm_device
    ng = P.ncol
    bounds = torch.tensor([block_range(P.nrow, q, i)[0] for i in range(1, q)], dtype=torch.int32, device=dev)
    col = torch.repeat_interleave(torch.arange(ng, device=dev), torch.diff(P.cp))
    blk = torch.bucketize(P.ir, bounds, right=True).to(torch.int64)
    key = blk * ng + col
    order = torch.argsort(key, stable=True)
    cnt = torch.bincount(key, minlength=q * ng).view(q, ng)
    starts = torch.tensor([block_range(P.nrow, q, i)[0] for i in range(q)], dtype=torch.int32, device=dev)
    s_ir = P.ir[order] - starts[blk[order]]
    s_val = P.val[order]
    send_nnz = [int(x) for x in cnt.sum(1).cpu().tolist()]
    send_n = torch.tensor(send_nnz, dtype=torch.int64, device=cd)
    recv_n = torch.empty(q, dtype=torch.int64, device=cd)
    dist.all_to_all_single(recv_n, send_n, group=grid.col_group)
    recv_nnz = [int(x) for x in recv_n.cpu().tolist()]
    col_split = [g1 - g0 for (g0, g1) in groups]
    r_cnt = torch.empty(sum(col_split), dtype=torch.int64, device=cd)
    r_ir = torch.empty(sum(recv_nnz), dtype=torch.int32, device=cd)
    r_val = torch.empty(sum(recv_nnz), dtype=be.val_dtype, device=cd)
    dist.all_to_all_single(r_cnt, _to_comm(cnt.reshape(-1), be), col_split, [ng] * q, group=grid.col_group)
    dist.all_to_all_single(r_ir, _to_comm(s_ir.to(torch.int32), be), recv_nnz, send_nnz, group=grid.col_group)
    dist.all_to_all_single(r_val, _to_comm(s_val, be), recv_nnz, send_nnz, group=grid.col_group)
    cp = torch.zeros(sum(col_split) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(_from_comm(r_cnt, be), 0, out=cp[1:])
    return Block(nrow_local, sum(col_split), cp, _from_comm(r_ir, be), _from_comm(r_val, be))


def MCLPruneRecoverySelect(A, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1):
    """Distributed prune/select/recover (ParFriends.h:185-353) of a colsplit SpParMat3D, in place.
    Columns are completed along the processor column (one all-to-all each way), pruned on device
    (backend.mcl_prune = cbg_mcl_prune), and returned.  Returns the global branch counts."""
    g, be = A.grid, A.backend
    if recoverPct > 1:
        recoverPct = recoverPct / 100.0
    if g.q == 1:
        P, st = be.mcl_prune(A.block, hardThreshold, selectNum, recoverNum, recoverPct)
        A.block = P
    else:
        full, groups = _gather_columns(A.block, g, A.nrow, be)
        P, st = be.mcl_prune(full, hardThreshold, selectNum, recoverNum, recoverPct)
        A.block = _scatter_columns(P, g, groups, A.block.nrow, be)
    t = torch.tensor([st["recovered"], st["selected"], st["recovered_after_select"]], dtype=torch.int64,
                     device=be.comm_device)
    dist.all_reduce(t)
    r = [int(x) for x in t.cpu().tolist()]
    return {"recovered": r[0], "selected": r[1], "recovered_after_select": r[2]}


def MemEfficientSpGEMM(SR, A, B, phases, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1,
                       computationKernel=1, perProcessMemory=0, stats=None):
    """HipMCL expansion (ParFriends.h:449-730): B's local columns are cut into `phases` pieces
    (ColSplit); each phase is a full SUMMA product A * B_p followed by MCLPruneRecoverySelect, and
    the pruned pieces are concatenated (ColConcatenate).  On a 3D grid (L > 1) the layer exchange
    would interleave phase pieces, so phases = 1 there (MemEfficientSpGEMM3D's own phasing is not
    mirrored); the product is phase-count independent either way."""
    g, be = A.grid, A.backend
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, "MemEfficientSpGEMM")
    if phases < 1 or phases >= A.ncol or g.L > 1:
        phases = 1
    ncl = B.block.ncol
    pieces = []
    counts = {"recovered": 0, "selected": 0, "recovered_after_select": 0}
    for p in range(phases):
        c0, c1 = block_range(ncl, phases, p)
        Bp = SpParMat3D(g, B.nrow, B.ncol, _col_slice(B.block, c0, c1) if phases > 1 else B.block, False, be)
        Cp = Mult_AnXBn_SUMMA3D(SR, A, Bp, stats)
        st = MCLPruneRecoverySelect(Cp, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion)
        for k in counts:
            counts[k] += st[k]
        pieces.append(Cp.block)
    blk = pieces[0] if phases == 1 else _col_concat(pieces, be.device)
    if stats is not None:
        stats.update(counts)
        stats["phases"] = phases
    return SpParMat3D(g, A.nrow, B.ncol, blk, True, be)


# -------------------------------------------------------------------------------------- backends
_TYPESTR = {torch.float64: "<f8", torch.float32: "<f4", torch.int64: "<i8", torch.int32: "<i4", torch.uint8: "|u1"}


class _ResultOwner:
    """Keeps a cbg_csc_result alive while torch tensors view its arrays."""

    def __init__(self, ctx, res):
        self.ctx, self.res, self.released = ctx, res, False

    def __del__(self):
        if not self.released and self.res is not None and self.res._owner:
            try:
                self.ctx._lib.cbg_result_free(self.ctx._ptr, ctypes.byref(self.res))
            except Exception:
                pass


class _DevArr:
    """1-D device array view for torch.as_tensor (__cuda_array_interface__, HIP device pointer)."""

    def __init__(self, ptr, n, typestr, owner):
        self.owner = owner
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr,
                                         "data": (int(ptr or 0), False), "version": 2, "strides": None}


class GpuBackend:
    """Local multiply / merge on the MI355X through libcbgpu; blocks live in HBM as torch tensors.
    libcbgpu runs on torch's current stream, so RCCL waits order against it."""

    def __init__(self, ctx, val_dtype=torch.float64):
        self.ctx = ctx
        self.device = torch.device("cuda", ctx.device)
        self.val_dtype = val_dtype
        # gloo moves CPU tensors only: stage through the host when the group is not RCCL
        self.comm_device = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
        # one stream shared by torch and libcbgpu: torch's default is the legacy NULL stream, which a
        # non-blocking library stream would not be ordered against
        self.stream = torch.cuda.Stream(self.device)
        torch.cuda.set_stream(self.stream)
        ctx.set_stream(self.stream.cuda_stream)

    def _view(self, b):
        return _abi.DcscView(b.nrow, b.ncol, b.nnz, b.ncol, b.cp.data_ptr(), None,
                             b.ir.data_ptr() if b.nnz else None, 4, 8,
                             b.val.data_ptr() if b.nnz else None, _ABI_DT[b.val.dtype], 1)

    def _res_view(self, b):
        r = _abi.CscResult()
        r.nrow, r.ncol, r.nnz = b.nrow, b.ncol, b.nnz
        r.colptr, r.row, r.val = b.cp.data_ptr(), (b.ir.data_ptr() if b.nnz else None), \
            (b.val.data_ptr() if b.nnz else None)
        r.val_type = _ABI_DT[b.val.dtype]
        return r

    def _take(self, res, kind="mul"):
        """Library result -> Block.  Zero-copy: torch tensors view the result's HBM arrays through
        __cuda_array_interface__ and keep an owner alive that frees the result (back into the
        context's caching pool) when the last tensor goes.  Falls back to a device copy."""
        owner = None
        zc = os.environ.get("CBG_ZERO_COPY", "1")
        if zc == "0" or (zc not in ("1", kind)):
            return self._copy(res)
        try:
            owner = _ResultOwner(self.ctx, res)
            n, nc = int(res.nnz), int(res.ncol)
            cp = torch.as_tensor(_DevArr(res.colptr, nc + 1, "<i8", owner), device=self.device)
            ir = torch.as_tensor(_DevArr(res.row, n, "<i4", owner), device=self.device)
            val = torch.as_tensor(_DevArr(res.val, n, _TYPESTR[self.val_dtype], owner), device=self.device)
            if cp.data_ptr() == res.colptr and (n == 0 or ir.data_ptr() == res.row):
                return Block(int(res.nrow), nc, cp, ir, val)
        except (TypeError, RuntimeError, ValueError):
            pass
        if owner is not None:
            owner.released = True   # not viewable zero-copy: the copy path frees the result
        return self._copy(res)

    def _copy(self, res):
        """Copy a library result into torch tensors (device-to-device) and release it."""
        lib = self.ctx._lib
        try:
            n, nc = int(res.nnz), int(res.ncol)
            cp = torch.empty(nc + 1, dtype=torch.int64, device=self.device)
            ir = torch.empty(n, dtype=torch.int32, device=self.device)
            val = torch.empty(n, dtype=self.val_dtype, device=self.device)
            _abi.check(lib.cbg_result_to_host(self.ctx._ptr, ctypes.byref(res), cp.data_ptr(),
                                              ir.data_ptr() if n else None, val.data_ptr() if n else None),
                       "cbg_result_to_host")
            return Block(int(res.nrow), nc, cp, ir, val)
        finally:
            lib.cbg_result_free(self.ctx._ptr, ctypes.byref(res))

    def multiply(self, A, B, sr, stats=None):
        lib = self.ctx._lib
        va, vb = self._view(A), self._view(B)
        res = _abi.CscResult()
        m = ctypes.c_int64(0)
        _abi.check(lib.cbg_spgemm_local(self.ctx._ptr, ctypes.byref(va), ctypes.byref(vb), sr.code, sr.dtype,
                                        _abi.SORTED_COLS, ctypes.byref(res), ctypes.byref(m)), "cbg_spgemm_local")
        if stats is not None:
            stats["multiplies"] = stats.get("multiplies", 0) + int(m.value)
        return self._take(res)

    def mcl_prune(self, blk, thr, select, recover, pct):
        res = _abi.CscResult()
        st = _abi.MclStats()
        _abi.check(self.ctx._lib.cbg_mcl_prune(self.ctx._ptr, ctypes.byref(self._res_view(blk)), float(thr),
                                               int(select), int(recover), float(pct), ctypes.byref(res),
                                               ctypes.byref(st)), "cbg_mcl_prune")
        return self._take(res, "merge"), {"recovered": st.recovered, "selected": st.selected,
                                          "recovered_after_select": st.recovered_after_select}

    def merge(self, parts, sr):
        arr = (_abi.CscResult * len(parts))(*[self._res_view(p) for p in parts])
        res = _abi.CscResult()
        _abi.check(self.ctx._lib.cbg_merge(self.ctx._ptr, arr, len(parts), sr.code, sr.dtype, _abi.SORTED_COLS,
                                           ctypes.byref(res)), "cbg_merge")
        return self._take(res, "merge")
