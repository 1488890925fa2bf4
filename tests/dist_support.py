"""TEST INFRASTRUCTURE for the distributed drivers (combblas_amd/dist.py).

`ScipyBackend` is a CPU stand-in for the local multiply/merge so that the SUMMA / 3D schedules, the
block distribution and the fiber exchange can be checked with gloo on CPU processes; it is never used
by the product.  `run_dist_case` is the per-rank body shared by the CPU (gloo + scipy) and GPU
(gloo + libcbgpu, ranks sharing cuda:0) tests: every rank builds the same global inputs, distributes
them, multiplies, and checks its own output piece against the global product.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from combblas_amd import dist as cbd  # noqa: E402
from combblas_amd.dist import Block  # noqa: E402


class ScipyBackend:
    """PlusTimes only (the schedules are semiring-agnostic; semirings are covered by the GPU tests)."""

    def __init__(self, val_dtype=torch.float64):
        self.device = torch.device("cpu")
        self.comm_device = torch.device("cpu")
        self.val_dtype = val_dtype

    @staticmethod
    def _csc(b):
        return sp.csc_matrix((b.val.numpy(), b.ir.numpy(), b.cp.numpy()), shape=(b.nrow, b.ncol))

    @staticmethod
    def _block(M, dtype):
        M = sp.csc_matrix(M)
        M.sum_duplicates()
        M.sort_indices()
        return Block(M.shape[0], M.shape[1], torch.as_tensor(M.indptr.astype(np.int64)),
                     torch.as_tensor(M.indices.astype(np.int32)), torch.as_tensor(M.data.astype(dtype)))

    def multiply(self, A, B, sr, stats=None):
        P = self._csc(A) @ self._csc(B)
        if stats is not None:
            m = int(np.diff(A.cp.numpy())[B.ir.numpy()].sum()) if B.nnz else 0
            stats["multiplies"] = stats.get("multiplies", 0) + m
        return self._block(P, A.val.numpy().dtype)

    def rmat_block(self, scale, edgefactor, seed, r0, r1, c0, c1):
        import combblas_amd as cb
        n, cp, ir, val = cb.generate_rmat_host(scale, edgefactor, seed=seed)   # host build of the same matrix
        lcp, lir, lval = cbd.slice_csc(cp, ir, val, r0, r1, c0, c1)
        return Block(r1 - r0, c1 - c0, torch.as_tensor(lcp), torch.as_tensor(lir), torch.as_tensor(lval))

    def mcl_prune(self, blk, thr, select, recover, pct):
        from helpers import Csc, oracle_mcl_prune
        P, st = oracle_mcl_prune(Csc(blk.nrow, blk.ncol, blk.cp.numpy(), blk.ir.numpy(), blk.val.numpy()),
                                 thr, select, recover, pct)
        return (Block(blk.nrow, blk.ncol, torch.as_tensor(P.cp), torch.as_tensor(P.ir), torch.as_tensor(P.val)),
                {"recovered": st[0], "selected": st[1], "recovered_after_select": st[2]})

    def merge(self, parts, sr):
        S = self._csc(parts[0])
        for p in parts[1:]:
            S = S + self._csc(p)
        return self._block(S, parts[0].val.numpy().dtype)


def random_csc(n, m, density, seed, dtype=np.float64, integer=True):
    rng = np.random.default_rng(seed)
    M = sp.random(n, m, density=density, format="csc", random_state=rng,
                  data_rvs=(lambda k: rng.integers(1, 5, k).astype(dtype)) if integer else None)
    M.sort_indices()
    return M


def init_group(rank, world, port, backend_kind):
    """torch process group of one test rank.  backend_kind:
      "scipy" / "gpu"  gloo; libcbgpu's grid runs over the host-staged gloo transport;
      "gpu-rccl"       nccl, one rank (RCCL refuses two ranks of one host on one device);
      "gpu-rccl-net"   gloo for the harness, libcbgpu's grid over its OWN RCCL communicators with every rank
                       on cuda:0: NCCL_HOSTID makes each rank its own RCCL "node", so RCCL's duplicate-GPU
                       check passes and its network (socket, loopback) transport carries the data.  The
                       broadcasts, grouped send/recv and all-gathers are the production RCCL calls on the
                       library's streams -- asynchronous, fenced by its HIP events -- not a stand-in."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend_kind == "gpu-rccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        return
    if backend_kind == "gpu-rccl-net":
        os.environ.update({"NCCL_HOSTID": f"cbg-test-rank-{rank}", "NCCL_SOCKET_IFNAME": "lo",
                           "NCCL_IB_DISABLE": "1", "CBG_GRID_TRANSPORT": "rccl"})
    dist.init_process_group("gloo", rank=rank, world_size=world)


def rccl_info(grid):
    """The cbg_grid_query record an RCCL grid of this shape must report."""
    return {"kind": "rccl", "ranks": {"world": grid.world, "row": grid.q, "col": grid.q, "fiber": grid.L}}


def run_dist_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body: init gloo, build the mandated grid for `world`, run every case."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        if backend_kind == "scipy":
            be = ScipyBackend()
        else:
            import combblas_amd as cb
            ctx = cb.Context(0)
            be = cbd.GpuBackend(ctx)
        for (n, k, m, dA, dB, seed) in cases:
            A = random_csc(n, k, dA, seed)
            B = random_csc(k, m, dB, seed + 1)
            Ad = cbd.SpParMat3D.from_global_csc(grid, n, k, A.indptr, A.indices, A.data, True, be)
            Bd = cbd.SpParMat3D.from_global_csc(grid, k, m, B.indptr, B.indices, B.data, False, be)
            stats = {}
            C = cbd.Mult_AnXBn_SUMMA3D(cb_sr(backend_kind), Ad, Bd, stats)
            R = (A @ B).tocsc()
            R.sort_indices()
            (r0, r1), (c0, c1) = C.local_range()
            Rl = R[r0:r1, c0:c1].tocsc()
            Rl.sort_indices()
            blk = C.block
            cp, ir, val = blk.cp.cpu().numpy(), blk.ir.cpu().numpy(), blk.val.cpu().numpy()
            assert (blk.nrow, blk.ncol) == (r1 - r0, c1 - c0), (blk.nrow, blk.ncol, r0, r1, c0, c1)
            assert np.array_equal(cp, Rl.indptr), f"rank {rank}: colptr differs"
            assert np.array_equal(ir, Rl.indices), f"rank {rank}: rows differ"
            assert np.array_equal(val, Rl.data), f"rank {rank}: values differ"   # integer-valued: exact
            # the layer multiplies add up to the product's multiplies
            t = torch.tensor([stats.get("multiplies", 0)], dtype=torch.int64)
            dist.all_reduce(t)
            want = int(np.diff(A.indptr)[B.indices].sum())
            assert int(t.item()) == want, (int(t.item()), want)
            assert C.getnnz() == R.nnz
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report to the parent, which fails the test
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def run_mcl_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body of the distributed HipMCL expansion (MemEfficientSpGEMM + prune): every rank
    checks its piece against the oracle's prune of the global product (complete columns)."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        if backend_kind == "scipy":
            be = ScipyBackend()
        else:
            import combblas_amd as cb
            be = cbd.GpuBackend(cb.Context(0))
        from combblas_amd.inputs import protein_like_graph
        from helpers import Csc, oracle_mcl_prune
        for (n, seed, phases, params) in cases:
            n, cp, ir, val = protein_like_graph(n, seed=seed, cmin=10, cmax=120, density=0.25, noise=1e-3)
            Ad = cbd.SpParMat3D.from_global_csc(grid, n, n, cp, ir, val, True, be)
            Bd = cbd.SpParMat3D.from_global_csc(grid, n, n, cp, ir, val, False, be)
            stats = {}
            C = cbd.MemEfficientSpGEMM(cb_sr(backend_kind), Ad, Bd, phases, *params, stats=stats)
            A = sp.csc_matrix((val, ir, cp), shape=(n, n))
            G = (A @ A).tocsc()
            G.sort_indices()
            O, ost = oracle_mcl_prune(Csc(n, n, G.indptr, G.indices, G.data), *params)
            R = sp.csc_matrix((O.val, O.ir, O.cp), shape=(n, n))
            (r0, r1), (c0, c1) = C.local_range()
            Rl = R[r0:r1, c0:c1].tocsc()
            Rl.sort_indices()
            blk = C.block
            assert np.array_equal(blk.cp.cpu().numpy(), Rl.indptr), f"rank {rank}: colptr differs"
            assert np.array_equal(blk.ir.cpu().numpy(), Rl.indices), f"rank {rank}: rows differ"
            assert np.allclose(blk.val.cpu().numpy(), Rl.data, rtol=1e-12, atol=0), f"rank {rank}: values"
            assert (stats["recovered"], stats["selected"], stats["recovered_after_select"]) == ost, (stats, ost)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def cb_sr(kind):
    import combblas_amd as cb
    return cb.PlusTimesSRing("f64")


def spawn_case(world, backend_kind, cases, port, body=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    procs = [ctx.Process(target=body or run_dist_case, args=(r, world, port, backend_kind, cases, errq)) for r in range(world)]
    for p in procs:
        p.start()
    # join with a heartbeat (a silent multi-minute wait looks hung to a watchdog) and a 300 s bound
    t0 = last = time.time()
    while any(p.is_alive() for p in procs) and time.time() - t0 < 300:
        time.sleep(0.2)
        if time.time() - last >= 30:
            last = time.time()
            alive = [r for r, p in enumerate(procs) if p.is_alive()]
            print(f"[spawn_case world={world}] {last - t0:.0f} s, ranks still running: {alive}",
                  file=sys.stderr, flush=True)
    for p in procs:
        p.join(timeout=1)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs and all(c == 0 for c in codes), "\n".join(errs) + f"\nexit codes {codes}"


def _check_piece(M, R, rank, what):
    """M's local piece (block distribution) equals the same block of the global scipy matrix R."""
    R = sp.csc_matrix(R)
    R.sum_duplicates()
    (r0, r1), (c0, c1) = M.local_range()
    Rl = R[r0:r1, c0:c1].tocsc()
    Rl.sort_indices()
    blk = M.block
    assert (M.nrow, M.ncol) == R.shape, (what, M.nrow, M.ncol, R.shape)
    assert (blk.nrow, blk.ncol) == (r1 - r0, c1 - c0), (what, blk.nrow, blk.ncol)
    assert np.array_equal(blk.cp.cpu().numpy(), Rl.indptr), f"rank {rank} {what}: colptr differs"
    assert np.array_equal(blk.ir.cpu().numpy(), Rl.indices), f"rank {rank} {what}: rows differ"
    assert np.array_equal(blk.val.cpu().numpy(), Rl.data), f"rank {rank} {what}: values differ"


def _pruned(A, ri, ci):
    """Global expectation of Prune: A without the entries (i, j), i in ri, j in ci."""
    C = sp.coo_matrix(A)
    drop = np.isin(C.row, ri) & np.isin(C.col, ci)
    return sp.csc_matrix((C.data[~drop], (C.row[~drop], C.col[~drop])), shape=A.shape)


def run_index_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body of the 2D drivers (Synch / DoubleBuff / Overlap) and of the SpGEMM-based
    indexing (SubsRef_SR, Prune, PruneFull, SpAsgn; SpParMat.cpp:2028-2562) on a one-layer grid."""
    try:
        init_group(rank, world, port, backend_kind)
        q = int(round(world ** 0.5))
        grid = cbd.CommGrid(q, q)
        if backend_kind == "scipy":
            be = ScipyBackend()
        else:
            import combblas_amd as cb
            be = cbd.GpuBackend(cb.Context(0))
        sr = cb_sr(backend_kind)
        for (n, m, density, seed) in cases:
            rng = np.random.default_rng(seed)
            A = random_csc(n, m, density, seed)
            B = random_csc(m, n, density, seed + 1)

            def dmat(M):
                return cbd.SpParMat3D.from_global_csc(grid, M.shape[0], M.shape[1], M.indptr, M.indices, M.data,
                                                      True, be)
            for f in (cbd.Mult_AnXBn_Synch, cbd.Mult_AnXBn_DoubleBuff, cbd.Mult_AnXBn_Overlap):
                _check_piece(f(sr, dmat(A), dmat(B)), A @ B, rank, f.__name__)
            ri = rng.integers(0, n, max(1, n // 3))          # duplicates allowed, unsorted
            ci = rng.permutation(m)[: max(1, m // 2)]
            _check_piece(cbd.SubsRef_SR(dmat(A), ri, ci), A[ri][:, ci], rank, "SubsRef_SR")
            _check_piece(dmat(A)(ri, ci), A[ri][:, ci], rank, "A(ri,ci)")
            _check_piece(cbd.SubsRef_SR_dim(dmat(A), ri, "row"), A[ri], rank, "SubsRef_SR row")
            _check_piece(cbd.SubsRef_SR_dim(dmat(A), ci, "column"), A[:, ci], rank, "SubsRef_SR column")
            D = dmat(A)
            cbd.SubsRef_SR(D, ri, ci, inplace=True)
            _check_piece(D, A[ri][:, ci], rank, "SubsRef_SR inplace")
            D = dmat(A)
            cbd.Prune(D, ri, ci)
            _check_piece(D, _pruned(A, ri, ci), rank, "Prune")
            D = dmat(A)
            cbd.PruneFull(D, ri, ci)
            Af = sp.coo_matrix(A)
            keep = ~(np.isin(Af.row, ri) | np.isin(Af.col, ci))
            _check_piece(D, sp.csc_matrix((Af.data[keep], (Af.row[keep], Af.col[keep])), shape=A.shape), rank,
                         "PruneFull")
            ru = rng.permutation(n)[: max(1, n // 4)]
            cu = rng.permutation(m)[: max(1, m // 3)]
            Bs = random_csc(ru.size, cu.size, 0.5, seed + 2)
            D = dmat(A)
            cbd.SpAsgn(D, ru, cu, dmat(Bs))
            Rm = sp.csc_matrix((np.ones(ru.size), (ru, np.arange(ru.size))), shape=(n, ru.size))
            Qm = sp.csc_matrix((np.ones(cu.size), (np.arange(cu.size), cu)), shape=(cu.size, m))
            _check_piece(D, _pruned(A, ru, cu) + Rm @ Bs @ Qm, rank, "SpAsgn")
            try:
                cbd.SubsRef_SR(dmat(A), [n], ci)
                raise AssertionError("out-of-range index accepted")
            except IndexError:
                pass
            try:
                cbd.SpAsgn(dmat(A), ru, cu, dmat(random_csc(ru.size + 1, cu.size, 0.5, seed)))
                raise AssertionError("SpAsgn dimension mismatch accepted")
            except Exception as e:
                assert getattr(e, "status", None) == 3002, e
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def _sr_obj(sr, dt):
    import combblas_amd as cb
    return {"plus_times": cb.PlusTimesSRing, "min_plus": cb.MinPlusSRing, "select2nd": cb.Select2ndSRing,
            "select_max": cb.SelectMaxSRing, "select_max_bool": cb.SelectMaxBoolSRing}[sr](dt)


def check_piece_exact_or_f64(M, R, rank, what, scale=None, rtol=1e-12):
    """M's local piece against the same block of the global CSC R (helpers.Csc or scipy): structure
    exact; values bit-exact, or |c - r| <= rtol * max(|r|, scale) when `scale` (a global scipy
    matrix of sum|a*b|) is given."""
    R = sp.csc_matrix(R)
    (r0, r1), (c0, c1) = M.local_range()
    Rl = R[r0:r1, c0:c1].tocsc()
    Rl.sort_indices()
    blk = M.block
    assert (blk.nrow, blk.ncol) == (r1 - r0, c1 - c0), (what, blk.nrow, blk.ncol)
    cp, ir, val = blk.cp.cpu().numpy(), blk.ir.cpu().numpy(), blk.val.cpu().numpy()
    assert np.array_equal(cp, Rl.indptr), f"rank {rank} {what}: colptr differs ({cp[-1]} vs {Rl.indptr[-1]})"
    assert np.array_equal(ir, Rl.indices), f"rank {rank} {what}: rows differ"
    if scale is None:
        assert np.array_equal(val.astype(np.float64), Rl.data.astype(np.float64)), f"rank {rank} {what}: values differ"
    else:
        S = sp.csc_matrix(scale)[r0:r1, c0:c1].tocsc()
        cols = np.repeat(np.arange(c1 - c0), np.diff(Rl.indptr))
        s = np.maximum(np.abs(Rl.data), np.asarray(S[Rl.indices, cols]).ravel())
        bad = np.abs(val - Rl.data) > rtol * s
        assert not bad.any(), f"rank {rank} {what}: {int(bad.sum())} values off"


def run_fixture_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body: the reference's own golden products (tests/golden, made by the reference-built
    refprobe) through the mandated layout for `world` (1x1x2, 2x2, 2x2x2), every semiring of the
    fixture, with Mult_AnXBn_SUMMA3D and -- on one-layer grids -- Synch / DoubleBuff / Overlap, and
    the 3DSpGEMM multiply (SUMMALayer + ReduceAll_threaded).  Each rank checks its own piece."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0)) if backend_kind.startswith("gpu") else ScipyBackend()
        from helpers import abs_product_sums, fixture_inputs, fixture_product, load_fixture
        for (name, tag, golden) in cases:
            z = load_fixture(name)
            A, B, sr, dt = fixture_inputs(z, tag)
            aval = A.val if A.val is not None else np.ones(A.nnz, np.uint8)
            Ad = cbd.SpParMat3D.from_global_csc(grid, A.nrow, A.ncol, A.cp, A.ir, aval, True, be)
            Bd = cbd.SpParMat3D.from_global_csc(grid, B.nrow, B.ncol, B.cp, B.ir, B.val, False, be)
            R = fixture_product(z, tag)
            Rs = sp.csc_matrix((R.val, R.ir, R.cp), shape=(A.nrow, B.ncol))
            scale = abs_product_sums(A, B) if dt == "f64" and sr == "plus_times" else None
            SR = _sr_obj(sr, dt)
            stats = {}
            drivers = [("SUMMA3D", lambda: cbd.Mult_AnXBn_SUMMA3D(SR, Ad, Bd, stats)),
                       ("multiply", lambda: cbd.multiply(SR, Ad, Bd))]
            if L == 1:
                drivers += [(f.__name__, (lambda f=f: f(SR, Ad, Bd)))
                            for f in (cbd.Mult_AnXBn_Synch, cbd.Mult_AnXBn_DoubleBuff, cbd.Mult_AnXBn_Overlap)]
            for dname, run in drivers:
                C = run()
                check_piece_exact_or_f64(C, Rs, rank, f"{name}/{tag}/{dname}", scale)
                if golden is not None:   # MATLAB's bcsstk01^2 (3DSpGEMM/matlab/C.mtx), as test_mpipspgemm
                    G = sp.csc_matrix((z[golden + "_val"], z[golden + "_ir"], z[golden + "_cp"]),
                                      shape=(A.nrow, B.ncol))
                    check_piece_exact_or_f64(C, G, rank, f"{name}/matlab/{dname}", scale)
            t = torch.tensor([stats.get("multiplies", 0)], dtype=torch.int64, device=be.comm_device)
            dist.all_reduce(t)
            assert int(t.item()) == int(z[f"C_{tag}_flops"]), (int(t.item()), int(z[f"C_{tag}_flops"]))
            if backend_kind.startswith("gpu-rccl"):   # RCCL itself counted the members of every group
                assert be.native_grid(grid).info() == rccl_info(grid), be.native_grid(grid).info()
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def run_block_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body of BlockSpGEMM / BlockSplit (BlockSpGEMM.h:14-130, SpParMat.cpp:2915-3000) and
    SpParMat3D::Convert2D (SpParMat3D.cpp:441-566) on the reference's G500 s10 fixture: every output
    block of A*A against the same block of the reference-built golden product, every BlockSplit piece
    against the slice of A, and Convert2D of colsplit / rowsplit 3D layouts against the 2D blocks."""
    try:
        init_group(rank, world, port, backend_kind)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0)) if backend_kind.startswith("gpu") else ScipyBackend()
        from helpers import fixture_inputs, fixture_product, load_fixture
        q = int(round(world ** 0.5))
        grid = cbd.CommGrid(q, q)
        z = load_fixture("g500_s10")
        A, B, sr, dt = fixture_inputs(z, "pt_f64_hash")
        R = fixture_product(z, "pt_f64_hash")
        As = sp.csc_matrix((A.val, A.ir, A.cp), shape=(A.nrow, A.ncol))
        Rs = sp.csc_matrix((R.val, R.ir, R.cp), shape=(A.nrow, B.ncol))
        SR = cb.PlusTimesSRing("f64")

        def dmat(M, colsplit=True, g=grid):
            return cbd.SpParMat3D.from_global_csc(g, M.shape[0], M.shape[1], M.indptr, M.indices, M.data, colsplit, be)
        for (br, bc) in cases:
            bs = cbd.BlockSpGEMM(dmat(As), dmat(As), br, bc)
            ro, co = bs.getBlockOffsets(True), bs.getBlockOffsets(False)
            assert ro[0] == 0 and ro[-1] == A.nrow and co[-1] == A.ncol and len(ro) == br + 1
            seen = 0
            while bs.hasNext():
                C, r0, c0 = bs.getNextBlock(SR)
                i, j = divmod(seen, bc)
                assert (r0, c0) == (ro[i], co[j]), (r0, c0, ro[i], co[j])
                _check_piece(C, Rs[ro[i]:ro[i + 1], co[j]:co[j + 1]], rank, f"BlockSpGEMM {br}x{bc} ({i},{j})")
                seen += 1
            assert seen == br * bc
            for i, row in enumerate(bs.A_blocks):
                _check_piece(row[0], As[ro[i]:ro[i + 1], :], rank, f"BlockSplit A {i}")
            C, r0, c0 = bs.getBlockId(SR, br - 1, bc - 1)
            _check_piece(C, Rs[ro[-2]:, co[-2]:], rank, "BlockSpGEMM getBlockId")
        for (L, qq) in ((world, 1), (1, q)):
            g3 = cbd.CommGrid3D(L, qq, qq)
            for colsplit in (True, False):
                M2 = cbd.Convert2D(dmat(Rs, colsplit, g3))
                _check_piece(M2, Rs, rank, f"Convert2D {L}x{qq}x{qq} colsplit={colsplit}")
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def run_rmat_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body: every rank builds only its own pieces of the reference's Graph500 Kronecker matrix
    (SpParMat3D.from_rmat -> cbg_rmat_block), which must equal the same blocks of the reference-generated
    matrix in the fixture, and the SUMMA3D product of those pieces must equal the reference's product."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0)) if backend_kind.startswith("gpu") else ScipyBackend()
        from helpers import fixture_product, load_fixture
        for (name, scale) in cases:
            if name in ("single-gpu", "fiber-mode"):   # the layouts against the one-GPU product of the same matrix
                Ad = cbd.SpParMat3D.from_rmat(grid, scale, 16, cb.G500_SEED, True, be)
                Bd = cbd.SpParMat3D.from_rmat(grid, scale, 16, cb.G500_SEED, False, be)
                st = {}
                C = cbd.Mult_AnXBn_SUMMA3D(cb.PlusTimesSRing("f64"), Ad, Bd, st)
                if name == "fiber-mode":   # the grid's two-layer fiber step: gather for A*A, unless switched off
                    want = "none" if L == 1 else ("reduce" if os.environ.get("CBG_FIBER_GATHER") == "0" else "gather")
                    got = st.get("fiber_mode", "none")
                    assert got == want, f"rank {rank}: fiber mode {got}, expected {want}"
                    if want == "gather":   # the operands crossed the fiber, not partial products
                        assert st["fiber_bytes"] > 0 and st["merge_ms"] == 0
                M = be.ctx.generate_rmat(scale, 16, seed=cb.G500_SEED)
                P = cb.LocalSpGEMMHash(cb.PlusTimesSRing("f64"), M, M)
                cp, ir, val = P.to_host()
                P.free()
                M.free()
                n = 1 << scale
                check_piece_exact_or_f64(C, sp.csc_matrix((val, ir, cp), shape=(n, n)), rank, f"s{scale} C piece")
                continue
            z = load_fixture(name)
            G = sp.csc_matrix((z["A_val"], z["A_ir"], z["A_cp"]), shape=tuple(z["A_shape"]))
            Ad = cbd.SpParMat3D.from_rmat(grid, scale, 16, cb.G500_SEED, True, be)
            Bd = cbd.SpParMat3D.from_rmat(grid, scale, 16, cb.G500_SEED, False, be)
            _check_piece(Ad, G, rank, f"{name} A piece")
            _check_piece(Bd, G, rank, f"{name} B piece")
            assert Ad.getnnz() == G.nnz
            if "C_pt_f64_hash_cp" in z.files:
                R = fixture_product(z, "pt_f64_hash")
            else:   # hashed fixture: the oracle's product, pinned to the reference's product hash
                from helpers import Csc, canonical_sha256, oracle_spgemm
                Ah = Csc(G.shape[0], G.shape[1], z["A_cp"], z["A_ir"], z["A_val"])
                R, _, rc = oracle_spgemm(Ah, Ah, "plus_times", "f64")
                assert rc == 0 and canonical_sha256(R.cp, R.ir, R.val) == str(z["C_pt_f64_hash_sha256"])
            C = cbd.Mult_AnXBn_SUMMA3D(cb.PlusTimesSRing("f64"), Ad, Bd)
            check_piece_exact_or_f64(C, sp.csc_matrix((R.val, R.ir, R.cp), shape=(G.shape[0], R.ncol)), rank,
                                     f"{name} C piece")
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def run_mcl_fixture_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body: the reference's MemEfficientSpGEMM output (tests/golden/mcl.npz, made by refprobe)
    through MemEfficientSpGEMM / MemEfficientSpGEMM3D on the mandated layout with phases 1..3: every
    phase count gives the reference's pruned product on every rank's piece and the same branch counts."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0)) if backend_kind.startswith("gpu") else ScipyBackend()
        from helpers import Csc, load_fixture, oracle_mcl_prune
        z = load_fixture("mcl")
        n = int(z["A_shape"][0])
        A = sp.csc_matrix((z["A_val"], z["A_ir"], z["A_cp"]), shape=(n, n))
        thr, sel, rec, pct = (float(x) for x in z["P1_params"])
        params = (thr, int(sel), int(rec), pct)
        G = (A @ A).tocsc()
        G.sort_indices()
        _, ost = oracle_mcl_prune(Csc(n, n, G.indptr, G.indices, G.data), *params)
        R = sp.csc_matrix((z["M1_val"], z["M1_ir"], z["M1_cp"]), shape=(n, n))
        S = (abs(A) @ abs(A)).tocsc()
        for case in cases:
            phases, mem = (1, case[1]) if isinstance(case, tuple) else (case, 0)
            Ad = cbd.SpParMat3D.from_global_csc(grid, n, n, z["A_cp"], z["A_ir"], z["A_val"], True, be)
            Bd = cbd.SpParMat3D.from_global_csc(grid, n, n, z["A_cp"], z["A_ir"], z["A_val"], False, be)
            stats = {}
            C = cbd.MemEfficientSpGEMM(cb.PlusTimesSRing("f64"), Ad, Bd, phases, *params, perProcessMemory=mem,
                                       stats=stats)
            if mem:   # a budget just above the inputs: the memory model must raise the phase count
                assert stats["phases"] > 1, stats
            else:
                assert stats["phases"] == phases, stats
            check_piece_exact_or_f64(C, R, rank, f"memeff phases={phases}", scale=S)
            assert (stats["recovered"], stats["selected"], stats["recovered_after_select"]) == ost, (stats, ost)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def run_galerkin_case(rank, world, port, backend_kind, cases, errq):
    """Per-rank body of the distributed Galerkin product (BASELINE config 5; RestrictionOp.cpp:155-196): with the
    reference's R (golden/galerkin.npz, made by refrestrict), R^T A and then (R^T A) R through the mandated layout
    for `world` -- Mult_AnXBn_SUMMA3D and the 3DSpGEMM multiply the reference's Galerkin driver calls -- and every
    rank's piece of both products against the reference's (refprobe LocalSpGEMMHash)."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0)) if backend_kind.startswith("gpu") else ScipyBackend()
        from helpers import load_fixture
        z = load_fixture("galerkin")
        n, nagg = (int(x) for x in z["R_shape"])
        PT = _sr_obj("plus_times", "f64")
        RT = cbd.SpParMat3D.from_global_csc(grid, nagg, n, z["RT_cp"], z["RT_ir"], z["RT_val"], True, be)
        A = cbd.SpParMat3D.from_global_csc(grid, n, n, z["A_cp"], z["A_ir"], z["A_val"], False, be)
        R = cbd.SpParMat3D.from_global_csc(grid, n, nagg, z["R_cp"], z["R_ir"], z["R_val"], False, be)
        gRA = sp.csc_matrix((z["RA_val"], z["RA_ir"], z["RA_cp"]), shape=(nagg, n))
        gC = sp.csc_matrix((z["C_val"], z["C_ir"], z["C_cp"]), shape=(nagg, nagg))
        if not backend_kind.startswith("gpu"):
            # scipy's product drops entries that cancel to 0.0; the reference (and libcbgpu) keep them
            # (returnedSAID() is false), so the CPU stand-in is compared with the fixture's zeros removed
            for M in (gRA, gC):
                M.eliminate_zeros()
        for name in cases:
            mult = cbd.Mult_AnXBn_SUMMA3D if name == "SUMMA3D" else cbd.multiply
            stats = {}
            RA = mult(PT, RT, A, stats) if name == "SUMMA3D" else mult(PT, RT, A)
            check_piece_exact_or_f64(RA, gRA, rank, f"galerkin/{name}/RtA", None)
            C = mult(PT, RA, R)
            check_piece_exact_or_f64(C, gC, rank, f"galerkin/{name}/RtAR", None)
            if name == "SUMMA3D":
                t = torch.tensor([stats.get("multiplies", 0)], dtype=torch.int64, device=be.comm_device)
                dist.all_reduce(t)
                assert int(t.item()) == int(z["RA_flops"]), (int(t.item()), int(z["RA_flops"]))
            if backend_kind.startswith("gpu-rccl"):
                assert be.native_grid(grid).info() == rccl_info(grid), be.native_grid(grid).info()
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def _values_csc(n, m, density, seed, kind):
    """Random CSC whose product exercises one fiber value format: 'small' (integers 1..4: varint, 1 byte),
    'wide' (integers up to 3000: products above 65535, varint of 2-4 bytes), 'huge' (integers ~2^20: products above
    2^32, neither varint nor f32 -> f64), 'real' (uniform reals: f64)."""
    rng = np.random.default_rng(seed)
    gen = {"small": lambda k: rng.integers(1, 5, k).astype(np.float64),
           "wide": lambda k: rng.integers(1, 3000, k).astype(np.float64),
           "huge": lambda k: rng.integers(1 << 20, 1 << 21, k).astype(np.float64),
           "real": lambda k: rng.random(k)}[kind]
    M = sp.random(n, m, density=density, format="csc", random_state=rng, data_rvs=gen)
    M.sort_indices()
    return M


def run_fiber_case(rank, world, port, backend_kind, cases, errq):
    """1x1x2 products whose fiber messages take every wire format (k_code_count picks per message): varint / 16-bit
    gap / int32 rows (dense runs, tall sparse columns with gaps above 2^14 and 2^16, columns of one chunk and of many),
    varint / u16 / f32 / f64 values; every rank's piece against scipy (exact for integer values, 1e-12 for reals),
    and the bytes on the wire reported by the grid stats within the bound of the format expected."""
    try:
        init_group(rank, world, port, backend_kind)
        L, q, _ = cbd.grid_for(world)
        grid = cbd.CommGrid3D(L, q, q)
        import combblas_amd as cb
        be = cbd.GpuBackend(cb.Context(0))
        for (n, k, m, dA, dB, seed, kind, max_bpe) in cases:
            A = _values_csc(n, k, dA, seed, kind)
            B = _values_csc(k, m, dB, seed + 1, kind)
            Ad = cbd.SpParMat3D.from_global_csc(grid, n, k, A.indptr, A.indices, A.data, True, be)
            Bd = cbd.SpParMat3D.from_global_csc(grid, k, m, B.indptr, B.indices, B.data, False, be)
            stats = {}
            C = cbd.Mult_AnXBn_SUMMA3D(cb_sr(backend_kind), Ad, Bd, stats)
            R = (A @ B).tocsc()
            R.sort_indices()
            (r0, r1), (c0, c1) = C.local_range()
            Rl = R[r0:r1, c0:c1].tocsc()
            Rl.sort_indices()
            blk = C.block
            assert np.array_equal(blk.cp.cpu().numpy(), Rl.indptr), f"rank {rank} {kind}: colptr differs"
            assert np.array_equal(blk.ir.cpu().numpy(), Rl.indices), f"rank {rank} {kind}: rows differ"
            v = blk.val.cpu().numpy()
            if kind == "real":
                assert np.allclose(v, Rl.data, rtol=1e-12, atol=0), f"rank {rank} {kind}: values differ"
            else:
                assert np.array_equal(v, Rl.data), f"rank {rank} {kind}: values differ"
            # what this rank sent: about half its layer partial (entries of the other layer's column half)
            t = torch.tensor([stats.get("fiber_bytes", 0), R.nnz], dtype=torch.float64)
            dist.all_reduce(t)
            if max_bpe is not None and R.nnz > 0:
                assert float(t[0]) <= max_bpe * R.nnz * 1.2 + 16 * m, (kind, float(t[0]), R.nnz)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise
