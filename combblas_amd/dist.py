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

    @classmethod
    def from_rmat(cls, grid, scale, edgefactor, seed, colsplit, backend):
        """This rank's piece of the reference's Graph500 Kronecker matrix, built on the rank's own device
        (DistEdgeList::GenGraph500Data(packed) + SpParMat(DEL), DistEdgeList.cpp:223-280,
        SpParMat.cpp:3082-3196; libcbgpu cbg_rmat_block).  The reference generates 1/p of the edges per
        rank and routes them to their owners with an all-to-all; every rank here replays the edge stream
        and keeps its own block, so no rank ever holds the global matrix and nothing is communicated."""
        n = 1 << int(scale)
        self = cls(grid, n, n, None, colsplit, backend)
        (r0, r1), (c0, c1) = self.local_range()
        self.block = backend.rmat_block(scale, edgefactor, seed, r0, r1, c0, c1)
        return self

    def __call__(self, ri, ci):
        """SpParMat::operator()(ri, ci) (SpParMat.h) = SubsRef_SR with PlusTimes semirings."""
        return SubsRef_SR(self, ri, ci)

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
def _row_slice(b, r0, r1):
    """Rows [r0, r1) of a Block, rebased (the row half of a transposed Split, SpDCCols.cpp:897)."""
    keep = (b.ir >= r0) & (b.ir < r1)
    cnt = torch.diff(b.cp)
    col = torch.repeat_interleave(torch.arange(b.ncol, device=b.cp.device), cnt)
    kc = torch.bincount(col[keep], minlength=b.ncol) if b.nnz else torch.zeros(b.ncol, dtype=torch.int64,
                                                                                  device=b.cp.device)
    cp = torch.zeros(b.ncol + 1, dtype=torch.int64, device=b.cp.device)
    torch.cumsum(kc, 0, out=cp[1:])
    return Block(r1 - r0, b.ncol, cp, (b.ir[keep] - r0).to(torch.int32), b.val[keep])


def _summa_partials(SR, A, B, stats, halves, running_merge=False):
    """The q SUMMA stages of one layer.  halves=False: one broadcast pair per stage; halves=True
    (Mult_AnXBn_DoubleBuff, ParFriends.h:799-997): every rank Splits its A piece by columns and its
    B piece by rows at half the inner width (SpDCCols::Split, cut = n/2) and the stages run once per
    half, so only half a stage's operands is in flight at a time.  Each stage's broadcasts are
    issued one stage ahead (async) so they overlap the current local multiply."""
    g, be = A.grid, A.backend
    q, L = g.q, g.L
    r0, r1 = block_range(A.nrow, q, g.row)
    ncl = B.block.ncol   # local columns of B (= of C): block `col` of B, or a phase piece of it
    widths = [piece_range(A.ncol, q, L, k, g.layer) for k in range(q)]
    widths = [k1 - k0 for (k0, k1) in widths]
    if halves:
        ca, cb = A.block.ncol // 2, B.block.nrow // 2   # this rank's A piece is inner block `col`, its B piece `row`
        mine = [(_col_slice(A.block, 0, ca), _row_slice(B.block, 0, cb)),
                (_col_slice(A.block, ca, A.block.ncol), _row_slice(B.block, cb, B.block.nrow))]
        spans = [[(w // 2) for w in widths], [w - w // 2 for w in widths]]
    else:
        mine = [(A.block, B.block)]
        spans = [widths]
    rounds = []
    for (ab, bb), sp_ in zip(mine, spans):
        a_nnz = _allgather_nnz(ab, g.row_group, q, be)   # pieces (l, i, k), k = 0..q-1
        b_nnz = _allgather_nnz(bb, g.col_group, q, be)   # pieces (l, k, j)
        rounds.append((ab, bb, sp_, a_nnz, b_nnz))

    def issue(h, k):
        ab, bb, sp_, a_nnz, b_nnz = rounds[h]
        a = _BlockBcast(ab, r1 - r0, sp_[k], a_nnz[k], g.rank_of(g.layer, g.row, k), g.row_group, be, g.rank)
        b = _BlockBcast(bb, sp_[k], ncl, b_nnz[k], g.rank_of(g.layer, k, g.col), g.col_group, be, g.rank)
        return a, b

    steps = [(h, k) for h in range(len(rounds)) for k in range(q)]
    partials = []
    pending = issue(*steps[0]) if q > 1 else None
    for s, (h, k) in enumerate(steps):
        if q > 1:
            a, b = pending
            Ak, Bk = a.wait(), b.wait()
            if s + 1 < len(steps):
                pending = issue(*steps[s + 1])   # double buffering: the next stage travels during this one
        else:
            Ak, Bk = rounds[h][0], rounds[h][1]
        if Ak.ncol == 0:   # an empty half (Split of a one-column piece): nothing to multiply
            partials.append(Block(r1 - r0, ncl, torch.zeros(ncl + 1, dtype=torch.int64, device=be.device),
                                  torch.zeros(0, dtype=torch.int32, device=be.device),
                                  torch.zeros(0, dtype=be.val_dtype, device=be.device)))
        else:
            partials.append(be.multiply(Ak, Bk, SR, stats))
        if running_merge and len(partials) == 2:   # Mult_AnXBn_Overlap: merge after every stage
            partials = [be.merge(partials, SR)] if partials[1].nnz else partials[:1]
    nonempty = [p for p in partials if p.nnz]
    return nonempty or partials[:1]


def _check_operands(A, B, name):
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, name)
    if not A.colsplit or B.colsplit or B.grid is not A.grid:
        raise ValueError("A must be colsplit and B rowsplit on the same CommGrid3D")


def Mult_AnXBn_SUMMA3D(SR, A, B, stats=None, halves=False, running_merge=False):
    """C = A * B over the semiring on the 3D grid (ParFriends.h:2918-3208).  A must be colsplit,
    B rowsplit, on the same grid; C comes back colsplit.  Dimension checks as CheckSpGEMMCompliance
    (ParFriends.h:160-181): a mismatch raises (the reference aborts with DIMMISMATCH 3002).

    On the GPU backend the whole schedule runs inside libcbgpu (cbg_spgemm_grid: RCCL broadcasts on a
    communication stream, device merges, fiber all-to-all); backends without a native grid (the CPU
    test backend) run the same schedule here in Python."""
    g = A.grid
    _check_operands(A, B, "Mult_AnXBn_SUMMA3D")
    be = A.backend
    if hasattr(be, "spgemm_grid"):
        flags = (_abi.HALVES if halves else 0) | (_abi.RUNNING_MERGE if running_merge else 0)
        C = be.spgemm_grid(g, A.block, B.block, SR, flags, stats)
        return SpParMat3D(g, A.nrow, B.ncol, C, True, be)
    partials = _summa_partials(SR, A, B, stats, halves, running_merge)
    C = partials[0] if len(partials) == 1 else be.merge(partials, SR)
    if g.L > 1:
        C = _fiber_exchange(C, g, be, SR)
    return SpParMat3D(g, A.nrow, B.ncol, C, True, be)


def SUMMALayer(SR, A, B, stats=None):
    """3DSpGEMM/SUMMALayer.h:24-97: the layer's q SUMMA stages, returning the unmerged stage products
    (Blocks; the reference's unreducedC list).  The reference hard-codes PlusTimes; any semiring here."""
    _check_operands(A, B, "SUMMALayer")
    be = A.backend
    if hasattr(be, "summa_layer"):
        return be.summa_layer(A.grid, A.block, B.block, SR, stats)
    return _summa_partials(SR, A, B, stats, False)


def ReduceAll_threaded(SR, unreducedC, A, B):
    """3DSpGEMM/Reductions.h:134-155: merge the stage products, then the fiber all-to-all of layer
    column parts and the merge of what arrives; returns C's colsplit piece on A's grid."""
    g, be = A.grid, A.backend
    if hasattr(be, "reduce_all"):
        C = be.reduce_all(g, unreducedC, SR)
    else:
        C = unreducedC[0] if len(unreducedC) == 1 else be.merge(unreducedC, SR)
        if g.L > 1:
            C = _fiber_exchange(C, g, be, SR)
    return SpParMat3D(g, A.nrow, B.ncol, C, True, be)


def _as_2d_operands(A, B, name):
    """On a one-layer grid the A-side and B-side distributions coincide (both are the q x q block
    distribution of SpParMat), so any two SpParMat3D on it can be multiplied as in the 2D drivers."""
    if A.grid.L != 1:
        raise ValueError(f"{name} needs a 2D (one-layer) grid")
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, name)
    return (SpParMat3D(A.grid, A.nrow, A.ncol, A.block, True, A.backend),
            SpParMat3D(B.grid, B.nrow, B.ncol, B.block, False, B.backend))


def Mult_AnXBn_Synch(SR, A, B, clearA=False, clearB=False, stats=None):
    """2D SUMMA (ParFriends.h:1004-1108) = the one-layer case of the 3D driver.  clearA/clearB drop
    the operands' local blocks after the product (the reference deletes them)."""
    a, b = _as_2d_operands(A, B, "Mult_AnXBn_Synch")
    C = Mult_AnXBn_SUMMA3D(SR, a, b, stats)
    _clear(A, clearA)
    _clear(B, clearB and B is not A)
    return C


def Mult_AnXBn_DoubleBuff(SR, A, B, clearA=False, clearB=False, stats=None):
    """ParFriends.h:799-997: 2D SUMMA with each operand Split in two along the inner dimension and
    2q stages (half the operand memory in flight); 2q partials merged.  Same product as Synch."""
    a, b = _as_2d_operands(A, B, "Mult_AnXBn_DoubleBuff")
    C = Mult_AnXBn_SUMMA3D(SR, a, b, stats, halves=True)
    _clear(A, clearA)
    _clear(B, clearB and B is not A)
    return C


def Mult_AnXBn_Overlap(SR, A, B, clearA=False, clearB=False, stats=None):
    """ParFriends.h:1110-1235: 2D SUMMA with the next stage's broadcasts in flight during the current
    local multiply (as in every driver here) and a running merge: the accumulated product is merged
    with each new stage product (:1187-1189), so at most two partials are alive."""
    a, b = _as_2d_operands(A, B, "Mult_AnXBn_Overlap")
    C = Mult_AnXBn_SUMMA3D(SR, a, b, stats, running_merge=True)
    _clear(A, clearA)
    _clear(B, clearB and B is not A)
    return C


def _clear(M, flag):
    if flag:
        M.block = Block(M.block.nrow, M.block.ncol, torch.zeros(M.block.ncol + 1, dtype=torch.int64,
                                                                device=M.block.cp.device),
                        M.block.ir[:0], M.block.val[:0])


def PSpGEMM(SR, A, B, stats=None):
    """SpParMat.h:451-464: the default distributed SpGEMM (Mult_AnXBn_Synch)."""
    return Mult_AnXBn_Synch(SR, A, B, stats=stats)


def multiply(SR, A, B, stats=None):
    """3DSpGEMM driver entry (Multiplier.h:10-61): SUMMALayer, then ReduceAll_threaded."""
    return ReduceAll_threaded(SR, SUMMALayer(SR, A, B, stats), A, B)


# --------------------------------------------------------------------------- indexing via SpGEMM
# SpParMat's indexing operations are SpGEMMs with 0/1 selection matrices (SpParMat.cpp:2028-2562):
# A(ri, ci) = P * A * Q with P(k, ri[k]) = 1 and Q(ci[k], k) = 1.  Index vectors are replicated
# numpy arrays here (the reference's FullyDistVec is distributed; each rank only needs the entries
# that land in its own block, which it selects locally -- the alltoallv that routes them in the
# reference, SpParMat.cpp:2083-2127, is not needed).  2D (one-layer) grids, like SpParMat.

def _sr_for(be, cls_name):
    import combblas_amd as cb
    code = {torch.float64: "f64", torch.float32: "f32", torch.int64: "i64", torch.int32: "i32",
            torch.uint8: "bool"}[be.val_dtype]
    return getattr(cb, cls_name)(code)


def _index_vector(v, bound, what):
    v = np.asarray(v, dtype=np.int64).reshape(-1)
    if v.size and (int(v.min()) < 0 or int(v.max()) >= bound):
        # the reference throws outofrangeexception for max > total (SpParMat.cpp:2051); an index equal
        # to the dimension would build an out-of-range selection matrix there, so it is rejected too
        raise IndexError(f"{what}: index out of range [0, {bound})")
    return v


def _selection(grid, be, nrow, ncol, rows, cols):
    """This rank's block of the nrow x ncol 0/1 matrix with ones at (rows[k], cols[k]); duplicate
    positions collapse to one entry (the matrices are bool-valued in the reference)."""
    (r0, r1), (c0, c1) = block_range(nrow, grid.q, grid.row), block_range(ncol, grid.q, grid.col)
    m = (rows >= r0) & (rows < r1) & (cols >= c0) & (cols < c1)
    nr, nc = r1 - r0, c1 - c0
    key = np.unique((cols[m] - c0) * max(nr, 1) + (rows[m] - r0))
    c, r = key // max(nr, 1), key % max(nr, 1)
    cp = np.zeros(nc + 1, np.int64)
    np.cumsum(np.bincount(c, minlength=nc), out=cp[1:])
    vals = np.ones(key.size, dtype=torch.empty(0, dtype=be.val_dtype).numpy().dtype)
    return SpParMat3D(grid, nrow, ncol, block_from_host(nr, nc, cp, r.astype(np.int32), vals, be.device), True, be)


def _keys(b):
    col = torch.repeat_interleave(torch.arange(b.ncol, device=b.cp.device), torch.diff(b.cp))
    return col, col * max(b.nrow, 1) + b.ir.to(torch.int64)


def _set_difference(blk, other):
    """SpParMat::SetDifference: drop the entries of blk whose (row, col) also appear in other."""
    if blk.nnz == 0 or other.nnz == 0:
        return blk
    col, ka = _keys(blk)
    _, kb = _keys(other)
    keep = ~torch.isin(ka, kb)
    cp = torch.zeros(blk.ncol + 1, dtype=torch.int64, device=blk.cp.device)
    torch.cumsum(torch.bincount(col[keep], minlength=blk.ncol), 0, out=cp[1:])
    return Block(blk.nrow, blk.ncol, cp, blk.ir[keep], blk.val[keep])


def SubsRef_SR(A, ri, ci, PTNTBOOL=None, PTBOOLNT=None, inplace=False):
    """A(ri, ci) (SpParMat.cpp:2028-2247): PA = P*A over PTBOOLNT, then (PA)*Q over PTNTBOOL (both
    Mult_AnXBn_DoubleBuff).  Default semirings PlusTimes on A's value type (the reference's
    operator() uses PlusTimesSRing<bool,NT>).  Returns a len(ri) x len(ci) matrix, or replaces A."""
    g, be = A.grid, A.backend
    ri = _index_vector(ri, A.nrow, "SubsRef_SR ri")
    ci = _index_vector(ci, A.ncol, "SubsRef_SR ci")
    PTBOOLNT = PTBOOLNT or _sr_for(be, "PlusTimesSRing")
    PTNTBOOL = PTNTBOOL or _sr_for(be, "PlusTimesSRing")
    P = _selection(g, be, ri.size, A.nrow, np.arange(ri.size, dtype=np.int64), ri)
    PA = Mult_AnXBn_DoubleBuff(PTBOOLNT, P, A, clearA=True)
    Q = _selection(g, be, A.ncol, ci.size, ci, np.arange(ci.size, dtype=np.int64))
    C = Mult_AnXBn_DoubleBuff(PTNTBOOL, PA, Q, clearA=True, clearB=True)
    if inplace:
        A.nrow, A.ncol, A.block = C.nrow, C.ncol, C.block
        return SpParMat3D(g, 0, 0, None, True, be)   # dummy, as the reference
    return C


def SubsRef_SR_dim(A, v, dim, PTNTBOOL=None, PTBOOLNT=None, inplace=False):
    """Row or column extraction (SpParMat.cpp:2251-2422): dim "row" -> A(v, :) = V*A over PTBOOLNT,
    dim "column" -> A(:, v) = A*V' over PTNTBOOL."""
    g, be = A.grid, A.backend
    if dim in ("row", "Row", 0):
        v = _index_vector(v, A.nrow, "SubsRef_SR row")
        V = _selection(g, be, v.size, A.nrow, np.arange(v.size, dtype=np.int64), v)
        C = Mult_AnXBn_DoubleBuff(PTBOOLNT or _sr_for(be, "PlusTimesSRing"), V, A, clearA=True)
    elif dim in ("column", "Column", 1):
        v = _index_vector(v, A.ncol, "SubsRef_SR column")
        V = _selection(g, be, A.ncol, v.size, v, np.arange(v.size, dtype=np.int64))
        C = Mult_AnXBn_DoubleBuff(PTNTBOOL or _sr_for(be, "PlusTimesSRing"), A, V, clearB=True)
    else:
        raise ValueError("dim must be 'row' or 'column'")
    if inplace:
        A.nrow, A.ncol, A.block = C.nrow, C.ncol, C.block
        return SpParMat3D(g, 0, 0, None, True, be)
    return C


def Prune(A, ri, ci):
    """Remove A[ri, ci] in place (SpParMat.cpp:2474-2514): SA = S*A over BoolCopy2nd, SAT = SA*T over
    BoolCopy1st with S = diag(ri), T = diag(ci), then SetDifference(SAT)."""
    g, be = A.grid, A.backend
    ri = _index_vector(ri, A.nrow, "Prune ri")
    ci = _index_vector(ci, A.ncol, "Prune ci")
    S = _selection(g, be, A.nrow, A.nrow, ri, ri)
    SA = Mult_AnXBn_DoubleBuff(_sr_for(be, "BoolCopy2ndSRing"), S, A, clearA=True)
    T = _selection(g, be, A.ncol, A.ncol, ci, ci)
    SAT = Mult_AnXBn_DoubleBuff(_sr_for(be, "BoolCopy1stSRing"), SA, T, clearA=True, clearB=True)
    A.block = _set_difference(A.block, SAT.block)


def PruneFull(A, ri, ci):
    """Remove every nonzero of the rows ri and of the columns ci (SpParMat.cpp:2521-2562)."""
    g, be = A.grid, A.backend
    ri = _index_vector(ri, A.nrow, "PruneFull ri")
    ci = _index_vector(ci, A.ncol, "PruneFull ci")
    S = _selection(g, be, A.nrow, A.nrow, ri, ri)
    SA = Mult_AnXBn_DoubleBuff(_sr_for(be, "BoolCopy2ndSRing"), S, A, clearA=True)
    T = _selection(g, be, A.ncol, A.ncol, ci, ci)
    AT = Mult_AnXBn_DoubleBuff(_sr_for(be, "BoolCopy1stSRing"), A, T, clearB=True)
    A.block = _set_difference(_set_difference(A.block, SA.block), AT.block)


def SpAsgn(A, ri, ci, B):
    """A(ri, ci) = B in place (SpParMat.cpp:2426-2467): Prune(ri, ci) makes the hole, B is embedded
    as R*B*Q over PlusTimes (R(ri[k], k) = 1, Q(k, ci[k]) = 1) and extend-added (+=)."""
    g, be = A.grid, A.backend
    if B.grid is not g:
        raise ValueError("SpAsgn: grids are not comparable")
    ri = _index_vector(ri, A.nrow, "SpAsgn ri")
    ci = _index_vector(ci, A.ncol, "SpAsgn ci")
    if B.nrow != ri.size or B.ncol != ci.size:
        raise _abi.CbgError(_abi.EDIM, "SpAsgn")   # DIMMISMATCH (SpParMat.cpp:2441-2450)
    Prune(A, ri, ci)
    pt = _sr_for(be, "PlusTimesSRing")
    R = _selection(g, be, A.nrow, B.nrow, ri, np.arange(ri.size, dtype=np.int64))
    RB = Mult_AnXBn_DoubleBuff(pt, R, B, clearA=True)
    Q = _selection(g, be, B.ncol, A.ncol, np.arange(ci.size, dtype=np.int64), ci)
    RBQ = Mult_AnXBn_DoubleBuff(pt, RB, Q, clearA=True, clearB=True)
    A.block = be.merge([A.block, RBQ.block], pt) if RBQ.block.nnz else A.block


# ------------------------------------------------------------------------------- block products
def _block_offsets(n, b):
    """BlockSpGEMM::getBlockOffsets / BlockSplit sizes (BlockSpGEMM.h:107-130, SpParMat.cpp:2943-2953):
    b blocks of n // b, the first n % b of them one larger (unlike the SpParMat distribution, which
    gives the remainder to the last block)."""
    sz, r = divmod(int(n), int(b))
    return [min(i, r) * (sz + 1) + (0 if i < r else i - r) * sz for i in range(b)] + [int(n)]


def BlockSplit(A, br, bc):
    """SpParMat::BlockSplit (SpParMat.cpp:2915-3000): the br x bc grid of sub-matrices of A, each a
    matrix of its own on A's process grid (block distribution of the sub-matrix's dimensions).  The
    reference routes tuples with an all-to-all (SparseCommon, no duplicates); here each block is
    A(rows, cols) through the SpGEMM selection of SubsRef_SR (exact for every value type: v * 1).
    br == bc == 1, or more blocks than rows / columns, returns [[A]] as the reference does."""
    if (br == 1 and bc == 1) or br > A.nrow or bc > A.ncol:
        return [[A]]
    if A.grid.L != 1:
        raise ValueError("BlockSplit: SpParMat (one-layer grid) only")
    ro, co = _block_offsets(A.nrow, br), _block_offsets(A.ncol, bc)
    out = []
    for i in range(br):
        rows = np.arange(ro[i], ro[i + 1], dtype=np.int64)
        Ai = A if br == 1 else SubsRef_SR_dim(A, rows, "row")
        out.append([Ai if bc == 1 else SubsRef_SR_dim(Ai, np.arange(co[j], co[j + 1], dtype=np.int64), "column")
                    for j in range(bc)])
    return out


class BlockSpGEMM:
    """C = A * B one output block at a time (BlockSpGEMM.h:14-130): A is split into br row blocks, B
    into bc column blocks (bi = 1: the inner dimension is not split, as the reference's getNextBlock
    asserts), and block (i, j) = Mult_AnXBn_DoubleBuff(A_i, B_j).  Python returns (C_ij, roffset,
    coffset) where the reference fills the two offsets by reference."""

    def __init__(self, A, B, br, bc, bi=1):
        self.br, self.bc, self.bi, self.cur = int(br), int(bc), int(bi), 0
        self.A_blocks = BlockSplit(A, self.br, self.bi)
        self.B_blocks = BlockSplit(B, self.bi, self.bc)
        self.nr, self.nc = A.nrow, B.ncol

    def _offsets(self, rbid, cbid):
        return _block_offsets(self.nr, self.br)[rbid], _block_offsets(self.nc, self.bc)[cbid]

    def getBlockId(self, SR, rbid, cbid):
        if self.bi != 1:
            raise ValueError("BlockSpGEMM: bi must be 1 (BlockSpGEMM.h:55)")
        if rbid >= len(self.A_blocks) or cbid >= len(self.B_blocks[0]):
            raise IndexError("BlockSpGEMM: more blocks than rows/columns (BlockSplit returned the whole matrix)")
        ro, co = self._offsets(rbid, cbid)
        return Mult_AnXBn_DoubleBuff(SR, self.A_blocks[rbid][0], self.B_blocks[0][cbid]), ro, co

    def getNextBlock(self, SR):
        rbid, cbid = divmod(self.cur, self.bc)
        self.cur += 1
        return self.getBlockId(SR, rbid, cbid)

    def hasNext(self):
        return self.cur < self.br * self.bc

    def getBlockOffsets(self, is_row):
        return _block_offsets(self.nr, self.br) if is_row else _block_offsets(self.nc, self.bc)


def Convert2D(A):
    """SpParMat3D::Convert2D, non-special layout (SpParMat3D.cpp:496-564): every local entry's global
    (row, col) (the layer-part offsets of the colsplit / rowsplit piece) is routed to its owner on the
    2D grid over all ranks, CommGrid(world, 0, 0) -- a square sqrt(p) x sqrt(p) grid (the reference's
    CommGrid aborts otherwise) -- with one all-to-all; the received entries form the local CSC."""
    g, be = A.grid, A.backend
    s = int(round(g.world ** 0.5))
    if s * s != g.world:
        raise ValueError(f"Convert2D: {g.world} processes do not form a square 2D grid (CommGrid.cpp:44-50)")
    g2 = CommGrid(s, s)
    (r0, r1), (c0, c1) = A.local_range()
    b = A.block
    dev, cd = be.device, be.comm_device
    col = torch.repeat_interleave(torch.arange(b.ncol, device=dev, dtype=torch.int64), torch.diff(b.cp)) + c0
    row = b.ir.to(torch.int64) + r0
    rstep, cstep = max(A.nrow // s, 1), max(A.ncol // s, 1)
    oi = torch.clamp(row // rstep, max=s - 1)   # SpParMat::Owner: last block takes the remainder
    oj = torch.clamp(col // cstep, max=s - 1)
    owner = oi * s + oj
    order = torch.argsort(owner, stable=True)
    send_n = torch.bincount(owner, minlength=g.world)
    sn = [int(x) for x in send_n.cpu().tolist()]
    recv_n = torch.empty(g.world, dtype=torch.int64, device=cd)
    dist.all_to_all_single(recv_n, _to_comm(send_n, be))
    rn = [int(x) for x in recv_n.cpu().tolist()]
    lr = (row - oi * rstep)[order]
    lc = (col - oj * cstep)[order]
    tot = sum(rn)
    r_r = torch.empty(tot, dtype=torch.int64, device=cd)
    r_c = torch.empty(tot, dtype=torch.int64, device=cd)
    r_v = torch.empty(tot, dtype=be.val_dtype, device=cd)
    dist.all_to_all_single(r_r, _to_comm(lr, be), rn, sn)
    dist.all_to_all_single(r_c, _to_comm(lc, be), rn, sn)
    dist.all_to_all_single(r_v, _to_comm(b.val[order], be), rn, sn)
    r_r, r_c, r_v = _from_comm(r_r, be), _from_comm(r_c, be), _from_comm(r_v, be)
    (q0, q1), (p0, p1) = block_range(A.nrow, s, g2.row), block_range(A.ncol, s, g2.col)
    nr, nc = q1 - q0, p1 - p0
    key = r_c * max(nr, 1) + r_r
    o = torch.argsort(key)
    cp = torch.zeros(nc + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.bincount(r_c, minlength=nc), 0, out=cp[1:])
    return SpParMat3D(g2, A.nrow, A.ncol, Block(nr, nc, cp, r_r[o].to(torch.int32), r_v[o]), True, be)


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


def _pad_cols(b, ncol, device):
    """Block b widened to `ncol` columns with empty columns appended."""
    if b.ncol == ncol:
        return b
    tail = b.cp[-1:].expand(ncol - b.ncol)
    return Block(b.nrow, ncol, torch.cat([b.cp, tail]), b.ir, b.val)


def EstPerProcessNnzSUMMA(A, B, hashEstimate=True):
    """Max over ranks of the nnz of this rank's unmerged SUMMA stage products (ParFriends.h:1242-1347):
    the symbolic pass of every stage product (estimateFLOP + estimateNNZ_Hash) summed over the q stages
    of the layer, MAX-reduced over the world.  (The reference's loop computes colnnzC per stage but never
    adds it to its total, so it returns 0 and its memory model never raises `phases`; the estimate here is
    the one the formula intends.)"""
    g, be = A.grid, A.backend
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, "EstPerProcessNnzSUMMA")
    _check_operands(A, B, "EstPerProcessNnzSUMMA")
    if hasattr(be, "summa_estimate"):   # libcbgpu: broadcasts + symbolic pass per stage, nothing materialised
        nnz = be.summa_estimate(g, A.block, B.block)[1]
    else:                               # CPU test backend: the stage products' nnz
        nnz = sum(P.nnz for P in _summa_partials(_PATTERN_SR(be), A, B, None, False))
    t = torch.tensor([nnz], dtype=torch.int64, device=be.comm_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def _PATTERN_SR(be):
    from . import PlusTimesSRing
    return PlusTimesSRing("f64" if be.val_dtype == torch.float64 else "f32")


def _phases_for_memory(A, B, phases, selectNum, recoverNum, perProcessMemory):
    """The phase count of MemEfficientSpGEMM3D's memory model (ParFriends.h:3243-3290): inputs (five copies
    of the largest layer piece), the layer's A*A estimate (two copies), the k-select buffers and the
    post-selection output against perProcessMemory GB; the MAX over the world, never below `phases`."""
    g, be = A.grid, A.backend
    p = g.q * g.q
    # bytes per stored nonzero in this implementation: int32 row + value (+ amortised colptr), the role of
    # the reference's sizeof(IU) * 2 + sizeof(NU)
    per_in = 4 * 2 + (8 if be.val_dtype == torch.float64 else 4)
    per_out = per_in
    t = torch.tensor([A.block.nnz], dtype=torch.int64, device=be.comm_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    input_mem = int(t.item()) * per_in * 5
    asq = EstPerProcessNnzSUMMA(A, B)
    asq_mem = asq * per_out * 2
    ncl = max(1, B.block.ncol)
    d = -(-int((asq // g.L) * p ** 0.5) // ncl)
    k = min(max(selectNum, recoverNum), d)
    post_nnz = -(-int((ncl // g.L) * k) // max(1, int(p ** 0.5)))
    remaining = perProcessMemory * 1e9 - input_mem - post_nnz * per_out * 2
    ksel_mem = ncl * k * (per_out - 8) * 3        # k-select buffers hold values only (sizeof(NUO) * 3)
    calc = int(-(-(asq_mem + ksel_mem) // remaining)) if remaining > 0 else -1
    # B's local width differs across grid columns (the last block takes the remainder), so `calc` is
    # MAX-reduced over the world: every rank must issue the same number of phases (the same collectives)
    t = torch.tensor([max(phases, calc)], dtype=torch.int64, device=be.comm_device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def MemEfficientSpGEMM(SR, A, B, phases, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1,
                       computationKernel=1, perProcessMemory=0, stats=None):
    """HipMCL expansion, MemEfficientSpGEMM (ParFriends.h:449-730) on one layer and MemEfficientSpGEMM3D
    (ParFriends.h:3214-3705) on L > 1 layers.  The rank's B columns are cut into the L layer chunks of
    the output column split (CalculateColSplitDistributionOfLayer, SpParMat3D.cpp:576-606) and every
    chunk into `phases` pieces (ColSplit, ParFriends.h:3315-3325); phase p multiplies the p-th piece of
    every chunk (layer SUMMA), sends piece m to layer m along the fiber, merges, prunes
    (MCLPruneRecoverySelect on the layer) and keeps only the pruned piece; the rank's pieces are
    concatenated in phase order.  Pieces are padded to one width so the fiber split falls on piece
    boundaries.  The pruned product does not depend on `phases`.  perProcessMemory > 0 raises `phases`
    by the reference's memory model."""
    g, be = A.grid, A.backend
    if A.ncol != B.nrow:
        raise _abi.CbgError(_abi.EDIM, "MemEfficientSpGEMM")
    if phases < 1 or phases >= B.ncol:
        phases = 1
    if perProcessMemory > 0:
        phases = max(1, min(_phases_for_memory(A, B, phases, selectNum, recoverNum, perProcessMemory),
                            max(1, B.ncol - 1)))
    L = g.L
    ncl = B.block.ncol
    chunks = [block_range(ncl, L, m) for m in range(L)]
    piece = [[(c0 + a, c0 + b) for (a, b) in (block_range(c1 - c0, phases, p) for p in range(phases))]
             for (c0, c1) in chunks]
    pieces = []
    counts = {"recovered": 0, "selected": 0, "recovered_after_select": 0}
    for p in range(phases):
        sel = [piece[m][p] for m in range(L)]
        W = max(b - a for (a, b) in sel)
        if L == 1 and phases == 1:
            Bb = B.block
        else:
            Bb = _col_concat([_pad_cols(_col_slice(B.block, a, b), W, be.device) for (a, b) in sel], be.device) \
                if L > 1 else _col_slice(B.block, *sel[0])
        Cp = Mult_AnXBn_SUMMA3D(SR, A, SpParMat3D(g, B.nrow, B.ncol, Bb, False, be), stats)
        mine = sel[g.layer]
        if L > 1 and Cp.block.ncol != mine[1] - mine[0]:
            Cp.block = _col_slice(Cp.block, 0, mine[1] - mine[0])   # drop the padding columns
        st = MCLPruneRecoverySelect(Cp, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion)
        for k in counts:
            counts[k] += st[k]
        pieces.append(Cp.block)
    blk = pieces[0] if len(pieces) == 1 else _col_concat(pieces, be.device)
    if stats is not None:
        stats.update(counts)
        stats["phases"] = phases
    return SpParMat3D(g, A.nrow, B.ncol, blk, True, be)


# -------------------------------------------------------------------------------------- backends
_TYPESTR = {torch.float64: "<f8", torch.float32: "<f4", torch.int64: "<i8", torch.int32: "<i4", torch.uint8: "|u1"}
_FROM_ABI = {v: k for k, v in _ABI_DT.items()}


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


def _dev_u8(ptr, n, device):
    """uint8 device tensor viewing n bytes at a HIP device pointer (no copy)."""
    return torch.as_tensor(_DevArr(ptr, n, "|u1", None), device=device)


class _NativeGrid:
    """libcbgpu's cbg_grid for one CommGrid3D.  RCCL: the library's own RCCL communicators (world +
    ncclCommSplit row/col/fiber; the unique id travels over the default torch group) -- the default on
    an nccl (RCCL) process group, and forced on any group by CBG_GRID_TRANSPORT=rccl (the one-GPU
    multi-rank tests run it under gloo).  CBG_GRID_TRANSPORT=torch, or a gloo group: a cbg_transport
    whose callbacks stage device buffers through the host and run the collective on the grid's torch
    process groups."""

    def __init__(self, grid, backend):
        self.lib = backend.ctx._lib
        self.grid, self.backend = grid, backend
        self.ptr = ctypes.c_void_p()
        L, q = grid.L, grid.q
        mode = os.environ.get("CBG_GRID_TRANSPORT", "auto")
        if mode not in ("auto", "rccl", "torch"):
            raise ValueError(f"CBG_GRID_TRANSPORT={mode!r}: expected auto, rccl or torch")
        use_rccl = mode == "rccl" or (mode == "auto" and dist.get_backend() == "nccl")
        if use_rccl:
            uid = torch.zeros(128, dtype=torch.uint8)
            if grid.rank == 0:
                buf = ctypes.create_string_buffer(128)
                _abi.check(self.lib.cbg_rccl_unique_id(buf), "cbg_rccl_unique_id")
                uid = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
            t = uid.to(backend.comm_device)
            dist.broadcast(t, src=0)
            raw = bytes(t.cpu().numpy().tobytes())
            idbuf = ctypes.create_string_buffer(raw, 128)
            _abi.check(self.lib.cbg_grid_create_rccl(backend.ctx._ptr, idbuf, grid.world, grid.rank, L, q, q,
                                                     ctypes.byref(self.ptr)), "cbg_grid_create_rccl")
            self.kind = "rccl"
        else:
            l, i, j = grid.layer, grid.row, grid.col
            self.groups = {_abi.GROUP_ROW: grid.row_group, _abi.GROUP_COL: grid.col_group,
                           _abi.GROUP_FIBER: grid.fiber_group, _abi.GROUP_WORLD: None}
            self.members = {_abi.GROUP_ROW: [grid.rank_of(l, i, c) for c in range(q)],
                            _abi.GROUP_COL: [grid.rank_of(l, r, j) for r in range(q)],
                            _abi.GROUP_FIBER: [grid.rank_of(m, i, j) for m in range(L)],
                            _abi.GROUP_WORLD: list(range(grid.world))}
            # nccl process groups move device tensors directly; gloo moves host tensors
            self.direct = dist.get_backend() == "nccl"
            self._cbs = (_abi.BCAST_FN(self._bcast), _abi.ALLTOALLV_FN(self._alltoallv),
                         _abi.ALLGATHER_FN(self._allgather))
            self.transport = _abi.Transport(None, *self._cbs, 0)
            _abi.check(self.lib.cbg_grid_create(backend.ctx._ptr, ctypes.byref(self.transport), grid.world, grid.rank,
                                                L, q, q, ctypes.byref(self.ptr)), "cbg_grid_create")
            self.kind = ("torch-nccl" if self.direct else "host-staged ") + ("" if self.direct else dist.get_backend())

    # -- transport callbacks (gloo): return 0 on success, never raise into C
    def _bcast(self, user, g, buf, nbytes, root):
        try:
            dev = self.backend.device
            t = _dev_u8(buf, nbytes, dev)
            src = self.members[g][root]
            if self.direct:
                dist.broadcast(t, src=src, group=self.groups[g])
            else:
                h = t.cpu() if src == self.grid.rank else torch.empty(nbytes, dtype=torch.uint8)
                dist.broadcast(h, src=src, group=self.groups[g])
                if src != self.grid.rank:
                    t.copy_(h)
            torch.cuda.current_stream(dev).synchronize()
            return 0
        except Exception as e:  # pragma: no cover - reported through CBG_ECOMM
            print(f"cbg transport bcast: {e!r}", flush=True)
            return 1

    def _alltoallv(self, user, g, send, sbytes, recv, rbytes):
        try:
            dev = self.backend.device
            P = len(self.members[g])
            sb = [int(sbytes[m]) for m in range(P)]
            rb = [int(rbytes[m]) for m in range(P)]
            where = dev if self.direct else torch.device("cpu")
            s = _dev_u8(send, sum(sb), dev) if sum(sb) else torch.empty(0, dtype=torch.uint8, device=dev)
            s = s.to(where)
            r = torch.empty(sum(rb), dtype=torch.uint8, device=where)
            dist.all_to_all_single(r, s, output_split_sizes=rb, input_split_sizes=sb, group=self.groups[g])
            if sum(rb):
                _dev_u8(recv, sum(rb), dev).copy_(r)
            torch.cuda.current_stream(dev).synchronize()
            return 0
        except Exception as e:  # pragma: no cover
            print(f"cbg transport alltoallv: {e!r}", flush=True)
            return 1

    def _allgather(self, user, g, send, recv, nbytes):
        try:
            P = len(self.members[g])
            where = self.backend.device if self.direct else torch.device("cpu")
            mine = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8).to(where)
            out = [torch.empty(nbytes, dtype=torch.uint8, device=where) for _ in range(P)]
            dist.all_gather(out, mine, group=self.groups[g])
            allb = torch.cat(out).cpu().numpy().tobytes()
            ctypes.memmove(recv, allb, nbytes * P)
            return 0
        except Exception as e:  # pragma: no cover
            print(f"cbg transport allgather: {e!r}", flush=True)
            return 1

    def info(self):
        """{"kind": "rccl" | caller transport, "ranks": {world, row, col, fiber}}: for RCCL the member
        counts RCCL itself reports for each communicator (ncclCommCount)."""
        gi = _abi.GridInfo()
        _abi.check(self.lib.cbg_grid_query(self.ptr, ctypes.byref(gi)), "cbg_grid_query")
        r = list(gi.ranks)
        return {"kind": "rccl" if gi.rccl else self.kind,
                "ranks": {"world": r[_abi.GROUP_WORLD], "row": r[_abi.GROUP_ROW], "col": r[_abi.GROUP_COL],
                          "fiber": r[_abi.GROUP_FIBER]}}

    def close(self):
        if self.ptr:
            self.lib.cbg_grid_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()


def _stats_update(stats, st):
    if stats is None:
        return
    stats["multiplies"] = stats.get("multiplies", 0) + int(st.multiplies)
    for k in ("bcast_bytes", "fiber_bytes", "bcast_ms", "local_ms", "merge_ms", "fiber_ms", "total_ms",
              "fiber_xfer_ms"):
        stats[k] = stats.get(k, 0) + getattr(st, k)
    stats["stages"] = stats.get("stages", 0) + int(st.stages)
    for k in ("heavy_ms",):
        stats[k] = stats.get(k, 0.0) + float(getattr(st, k))
    for k in ("heavy_multiplies", "heavy_nnz_b", "heavy_nnz_c", "local_nnz_out", "local_nnz_b", "local_ncol_b",
              "local_products"):
        stats[k] = stats.get(k, 0) + int(getattr(st, k))
    # the two-layer fiber step the grid took (cbg_grid_stats.fiber_mode): a name, so per-step sums skip it
    if int(st.fiber_mode):
        stats["fiber_mode"] = {1: "reduce", 2: "gather"}.get(int(st.fiber_mode), str(int(st.fiber_mode)))


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
            vdt = _FROM_ABI.get(int(res.val_type), self.val_dtype)   # the result's own value type
            cp = torch.as_tensor(_DevArr(res.colptr, nc + 1, "<i8", owner), device=self.device)
            ir = torch.as_tensor(_DevArr(res.row, n, "<i4", owner), device=self.device)
            val = torch.as_tensor(_DevArr(res.val, n, _TYPESTR[vdt], owner), device=self.device)
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
            val = torch.empty(n, dtype=_FROM_ABI.get(int(res.val_type), self.val_dtype), device=self.device)
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

    def rmat_block(self, scale, edgefactor, seed, r0, r1, c0, c1):
        res = _abi.CscResult()
        _abi.check(self.ctx._lib.cbg_rmat_block(self.ctx._ptr, int(scale), int(edgefactor), int(seed), int(r0), int(r1),
                                                int(c0), int(c1), ctypes.byref(res)), "cbg_rmat_block")
        return self._take(res)

    def mcl_prune(self, blk, thr, select, recover, pct):
        res = _abi.CscResult()
        st = _abi.MclStats()
        _abi.check(self.ctx._lib.cbg_mcl_prune(self.ctx._ptr, ctypes.byref(self._res_view(blk)), float(thr),
                                               int(select), int(recover), float(pct), ctypes.byref(res),
                                               ctypes.byref(st)), "cbg_mcl_prune")
        return self._take(res, "merge"), {"recovered": st.recovered, "selected": st.selected,
                                          "recovered_after_select": st.recovered_after_select}

    # ------------------------------------------------------------------ native grid (cbg_grid)
    def native_grid(self, grid):
        key = id(grid)
        if not hasattr(self, "_grids"):
            self._grids = {}
        if key not in self._grids:
            self._grids[key] = (grid, _NativeGrid(grid, self))   # keep grid alive with its handle
        return self._grids[key][1]

    def spgemm_grid(self, grid, A, B, sr, flags=0, stats=None):
        ng = self.native_grid(grid)
        va, vb = self._view(A), self._view(B)
        res, st = _abi.CscResult(), _abi.GridStats()
        _abi.check(self.ctx._lib.cbg_spgemm_grid(ng.ptr, ctypes.byref(va), ctypes.byref(vb), sr.code, sr.dtype,
                                                 _abi.SORTED_COLS | flags, ctypes.byref(res), ctypes.byref(st)),
                   "cbg_spgemm_grid")
        _stats_update(stats, st)
        return self._take(res)

    def summa_layer(self, grid, A, B, sr, stats=None):
        ng = self.native_grid(grid)
        va, vb = self._view(A), self._view(B)
        parts = (_abi.CscResult * (2 * grid.q))()
        n, st = ctypes.c_int32(0), _abi.GridStats()
        _abi.check(self.ctx._lib.cbg_summa_layer(ng.ptr, ctypes.byref(va), ctypes.byref(vb), sr.code, sr.dtype,
                                                 _abi.SORTED_COLS, parts, ctypes.byref(n), ctypes.byref(st)),
                   "cbg_summa_layer")
        _stats_update(stats, st)
        out = []
        for k in range(n.value):
            r = _abi.CscResult()
            ctypes.pointer(r)[0] = parts[k]
            out.append(self._take(r))
        return out

    def summa_estimate(self, grid, A, B):
        """(multiplies, nnz) of this rank's unmerged stage products: symbolic passes only (cbg_summa_estimate)."""
        ng = self.native_grid(grid)
        va, vb = self._view(A), self._view(B)
        f, z = ctypes.c_int64(0), ctypes.c_int64(0)
        _abi.check(self.ctx._lib.cbg_summa_estimate(ng.ptr, ctypes.byref(va), ctypes.byref(vb), ctypes.byref(f),
                                                    ctypes.byref(z)), "cbg_summa_estimate")
        return int(f.value), int(z.value)

    def reduce_all(self, grid, parts, sr, stats=None):
        ng = self.native_grid(grid)
        arr = (_abi.CscResult * len(parts))(*[self._res_view(p) for p in parts])
        res, st = _abi.CscResult(), _abi.GridStats()
        _abi.check(self.ctx._lib.cbg_reduce_all(ng.ptr, arr, len(parts), sr.code, sr.dtype, ctypes.byref(res),
                                                ctypes.byref(st)), "cbg_reduce_all")
        _stats_update(stats, st)
        return self._take(res)

    def estimate(self, A, B):
        """(multiplies, nnz(C)) of A*B from the symbolic pass alone (cbg_estimate: estimateFLOP + exact nnz)."""
        va, vb = self._view(A), self._view(B)
        f, z = ctypes.c_int64(0), ctypes.c_int64(0)
        _abi.check(self.ctx._lib.cbg_estimate(self.ctx._ptr, ctypes.byref(va), ctypes.byref(vb), ctypes.byref(f),
                                              ctypes.byref(z)), "cbg_estimate")
        return int(f.value), int(z.value)

    def fiber_codec(self, P, chunks=2):
        """The production fiber encoder + decoder on partial P (cbg_fiber_codec): wire bytes per part and whether
        every chunk round-trips bit for bit."""
        st = _abi.CodecStats()
        _abi.check(self.ctx._lib.cbg_fiber_codec(self.ctx._ptr, ctypes.byref(self._res_view(P)), int(chunks),
                                                 ctypes.byref(st)), "cbg_fiber_codec")
        return {k: getattr(st, k) for k, _ in _abi.CodecStats._fields_}

    def merge(self, parts, sr):
        arr = (_abi.CscResult * len(parts))(*[self._res_view(p) for p in parts])
        res = _abi.CscResult()
        _abi.check(self.ctx._lib.cbg_merge(self.ctx._ptr, arr, len(parts), sr.code, sr.dtype, _abi.SORTED_COLS,
                                           ctypes.byref(res)), "cbg_merge")
        return self._take(res, "merge")
