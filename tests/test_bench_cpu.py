"""bench.py's host helpers on CPU tensors: the rank-share panels (A pieces side by side, B pieces stacked by rows,
as grid.hip's panel_cols / panel_rows lay them out), the fiber wire-byte count, the evidence-file order and the
entry checksum shared with oracle/ref/refbench.cpp, and tools/predict_scaling.py's step model."""
import os

import numpy as np
import scipy.sparse as sp
import torch

import bench
from combblas_amd import dist as cbd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _block(M):
    M = sp.csc_matrix(M)
    M.sort_indices()
    return cbd.Block(M.shape[0], M.shape[1], torch.as_tensor(M.indptr.astype(np.int64)),
                     torch.as_tensor(M.indices.astype(np.int32)), torch.as_tensor(M.data.astype(np.float64)))


def _dense(b):
    return sp.csc_matrix((b.val.numpy(), b.ir.numpy(), b.cp.numpy()), shape=(b.nrow, b.ncol)).toarray()


def test_panels_match_scipy_stacking():
    rng = np.random.default_rng(7)
    parts = [sp.random(50, 30 + k, density=0.1, random_state=rng) for k in range(3)]
    H = bench._hcat([_block(p) for p in parts])
    assert np.array_equal(_dense(H), sp.hstack(parts).toarray())
    parts = [sp.random(20 + k, 40, density=0.15, random_state=rng) for k in range(3)]
    V = bench._vstack([_block(p) for p in parts])
    assert np.array_equal(_dense(V), sp.vstack(parts).toarray())
    assert all(np.all(np.diff(V.ir.numpy()[V.cp[c]:V.cp[c + 1]]) > 0) for c in range(V.ncol))
    S = bench._col_slice_block(V, 5, 17)
    assert np.array_equal(_dense(S), sp.vstack(parts).toarray()[:, 5:17])


def test_fiber_wire_bytes_counts_gaps_escapes_and_values():
    # column 0: rows 3, 70000 (gap 69997 escapes), 70001; column 1 empty; column 2: dense run 100..163
    rows = [3, 70000, 70001] + list(range(100, 164))
    cp = [0, 3, 3, 67]
    vals = [1.0, 2.0, 300.0] + [1.0] * 64
    b = cbd.Block(80000, 3, torch.tensor(cp, dtype=torch.int64), torch.tensor(rows, dtype=torch.int32),
                  torch.tensor(vals, dtype=torch.float64))
    w = bench.fiber_wire_bytes(b)
    assert w["escapes"] == 1
    assert w["row_bytes"] == {"int32": 4 * 67, "gap16": 2 * 67 + 4, "varint": 1 + 3 + 1 + 1 + 63}
    assert w["value_bytes"]["u16"] == 2 * 67 and w["value_bytes"]["varint"] == 66 + 2 + 8 * 3
    assert (w["rows"], w["values"]) == ("varint", "varint")
    assert w["bytes"] == 8 * 3 + 69 + 92
    # the same accounting in column chunks (bounded temporaries for billions of entries) adds up the same
    c = bench.fiber_wire_bytes(b, chunk=4)
    assert (c["row_bytes"], c["rows"], c["values"], c["escapes"]) == (w["row_bytes"], "varint", "varint", 1)
    assert c["value_bytes"]["varint"] == 66 + 2 + 8 * 3 and c["bytes"] == w["bytes"]


def test_round_tag_orders_evidence_files():
    names = ["profiles/r03y_pmc_heavy.json", "profiles/r03aj_pmc_heavy.json", "profiles/r02zf_pmc_heavy.json",
             "profiles/r04b_pmc_heavy.json", "profiles/r03z_pmc_heavy.json"]
    assert sorted(names, key=bench.round_tag)[-2:] == ["profiles/r03aj_pmc_heavy.json", "profiles/r04b_pmc_heavy.json"]
    assert sorted(names, key=bench.round_tag)[0] == "profiles/r02zf_pmc_heavy.json"


def test_entry_checksum_is_order_independent():
    cp = np.array([0, 2, 3], np.int64)
    ir = np.array([1, 5, 0], np.int32)
    val = np.array([1.0, 2.0, 3.0])
    a = bench.entry_checksum(cp, ir, val)
    # same entries, rows of column 0 swapped: a different CSC order, the same multiset
    assert a == bench.entry_checksum(cp, np.array([5, 1, 0], np.int32), np.array([2.0, 1.0, 3.0]))
    assert a != bench.entry_checksum(cp, ir, np.array([1.0, 2.0, 4.0]))


def test_predict_scaling_model():
    """tools/predict_scaling.py: a fast link hides the fiber behind the own half, a slow one exposes it (less with
    more chunks); one-layer layouts pay broadcasts and one product only."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("predict_scaling", os.path.join(ROOT, "tools", "predict_scaling.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    ph = [{"total_ms": 50.0}, {"total_ms": 50.0}]
    r2 = {"rank": 0, "layout": "2x1x1", "scale": 21, "nnz_A_panel": 10, "nnz_B_panel": 10, "phases_ms": ph,
          "fiber": {"bytes": 5e9}, "recv_nnz": 0, "merge_ms": 20.0, "multiplies": 1e10}
    fast = ps.predict([r2], link_gbps=1000.0)
    assert fast["parts_ms"]["fiber_exposed"] == 0.0 and abs(fast["step_ms"] - 121.0) < 0.5
    slow2 = ps.predict([r2], link_gbps=50.0, chunks=2)["parts_ms"]["fiber_exposed"]
    slow4 = ps.predict([r2], link_gbps=50.0, chunks=4)["parts_ms"]["fiber_exposed"]
    assert slow2 > slow4 > 0   # 5 GB at 50 GB/s = 100 ms against 75 ms of compute after the first chunk
    r4 = {"rank": 0, "layout": "1x2x2", "scale": 21, "nnz_A_panel": 1e7, "nnz_B_panel": 1e7,
          "phases_ms": [{"total_ms": 55.0}], "fiber": None, "merge_ms": 0.0, "multiplies": 5e9}
    p4 = ps.predict([r4, dict(r4, rank=1)], link_gbps=60.0)
    assert p4["parts_ms"]["merge"] == 0.0 and abs(p4["parts_ms"]["bcast"] - 2.0) < 1e-6   # 120 MB at 60 GB/s
    assert p4["multiplies"] == 1e10


def test_select_block_cols_and_torch_checksum():
    """bench.py's distributed checks: a column sample of a Block, and the checksum of a piece's reference-sample
    columns summed over pieces equal to the checksum of the whole sample (what refbench prints)."""
    rng = np.random.default_rng(3)
    M = sp.random(40, 30, density=0.2, random_state=rng, format="csc")
    M.data = np.round(M.data * 100)
    b = _block(M)
    cols = torch.tensor([0, 3, 4, 17, 29])
    S = bench.select_block_cols(b, cols)
    assert np.array_equal(_dense(S), M.toarray()[:, cols.numpy()])
    stride = 3
    whole = M[:, ::stride].tocsc()
    whole.sort_indices()
    ref = bench.entry_checksum(whole.indptr.astype(np.int64), whole.indices.astype(np.int32), whole.data)
    total = 0
    for (r0, r1) in ((0, 25), (25, 40)):
        for (c0, c1) in ((0, 11), (11, 30)):
            P = sp.csc_matrix(M[r0:r1, c0:c1])
            P.sort_indices()
            first = (-c0) % stride
            jl = torch.arange(first, c1 - c0, stride)
            R = bench.select_block_cols(_block(P), jl)
            cc = torch.repeat_interleave((jl + c0) // stride, torch.diff(R.cp))
            total += bench.entry_checksum_t(cc, R.ir.to(torch.int64) + r0, R.val)
    assert f"{total & ((1 << 64) - 1):016x}" == ref


def test_host_cores_record():
    threads, rec = bench.host_cores(1)
    assert 1 <= threads <= 16 and threads <= rec["affinity_cpus"]
    assert rec["os_cpu_count"] == os.cpu_count() and rec["pool_share_cpus"] == 16


def test_piece_checksum_matches_entry_checksum():
    """bench.piece_checksum (device-side, column chunks, global ids) equals entry_checksum of the same entries: the
    per-rank sums of the distributed line add up to one whole-product checksum whatever the layout."""
    import numpy as np
    import torch
    import bench
    from combblas_amd import dist as cbd
    rng = np.random.default_rng(1)
    n, m = 50, 40
    cols = [np.sort(rng.choice(n, rng.integers(0, 8), replace=False)) for _ in range(m)]
    cp = np.r_[0, np.cumsum([len(c) for c in cols])].astype(np.int64)
    ir = np.concatenate(cols).astype(np.int32)
    val = rng.integers(1, 9, len(ir)).astype(np.float64)
    r0, c0 = 7, 11
    got = bench.piece_checksum(cbd.Block(n, m, torch.tensor(cp), torch.tensor(ir), torch.tensor(val)), r0, c0, chunk=5)
    # the same entries as one CSC with the global ids: rows + r0 in an (n + r0)-row matrix, columns shifted by c0
    gcp = np.r_[np.zeros(c0, np.int64), cp]
    assert f"{got & ((1 << 64) - 1):016x}" == bench.entry_checksum(gcp, ir.astype(np.int64) + r0, val)
    # split into two column pieces: the checksums add (mod 2^64)
    a = bench.piece_checksum(cbd.Block(n, 25, torch.tensor(cp[:26]), torch.tensor(ir[:cp[25]]),
                                       torch.tensor(val[:cp[25]])), r0, c0)
    b = bench.piece_checksum(cbd.Block(n, 15, torch.tensor(cp[25:] - cp[25]), torch.tensor(ir[cp[25]:]),
                                       torch.tensor(val[cp[25]:])), r0, c0 + 25)
    assert (a + b) & ((1 << 64) - 1) == got & ((1 << 64) - 1)


def _run_bench(args, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def test_bench_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two fresh rank processes itself (no GPU call in the
    launcher), rank 0's JSON line is the only stdout line, and the line is the launched world's (n_gpus 2)."""
    import json
    r = _run_bench(["--gpus", "2", "--launch-probe", "--no-cpu", "--scale", "8"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"] == 2 and d["rank_sum"] == 1.0
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1] and {x["world"] for x in d["ranks"]} == {2}
    assert sorted(x["local_rank"] for x in d["ranks"]) == [0, 1]
    assert len({x["pid"] for x in d["ranks"]}) == 2


def test_bench_launcher_fails_when_a_rank_fails():
    r = _run_bench(["--gpus", "2", "--launch-probe"], {"CBG_LAUNCH_PROBE_FAIL_RANK": "1"})
    assert r.returncode == 7, (r.returncode, r.stderr[-3000:])
    assert "rank 1 exited with status 7" in r.stderr


def test_bench_refuses_world_size_mismatch():
    r = _run_bench(["--gpus", "8", "--launch-probe"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_refuses_more_ranks_than_gpus_for_rccl():
    """With fewer visible GPUs than --gpus and the production backend, the launcher refuses (no silent sharing)."""
    r = _run_bench(["--gpus", "4"], {"CBG_DIST_BACKEND": "nccl", "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0 and "visible GPUs" in r.stderr
