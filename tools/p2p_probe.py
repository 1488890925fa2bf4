#!/usr/bin/env python3
"""xGMI point-to-point bandwidth probe for the driver's 8-GPU node: the link figure tools/predict_scaling.py assumes
(--link-GBps) becomes a measurement.

  python tools/p2p_probe.py [--mib 1024] [--reps 5] [--out profiles/<tag>_p2p_probe.json]

Two measurements per GPU pair (0, j), j = 1 .. N-1:
  copy    peer copies from GPU 0 to GPU j (one process, torch tensors, hipMemcpyPeer over xGMI): one direction, and
          both directions at once (two streams);
  rccl    the fiber exchange's own transport: two ranks (GPU 0 and GPU j, torch.distributed "nccl" = RCCL) exchanging
          one message each way with a grouped send/recv (ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd, as
          grid.hip's fiber pipeline posts them), timed between barriers.
Prints one JSON object (GB/s per pair and direction; `link_GBps` = the median one-direction RCCL rate, what the step
model takes) and writes it to --out.  Needs >= 2 visible GPUs; on fewer it prints why and exits 0 (nothing to
measure).  The RCCL pairs run as fresh child processes started before this process touches a GPU."""
import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def rccl_pair(args):
    """Child: rank r of a 2-rank RCCL group on GPU (0, peer)[r]; one grouped exchange of --mib each way, timed."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    dev = 0 if rank == 0 else args.peer
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    n = args.mib << 20
    send = torch.ones(n, dtype=torch.uint8, device=dev)
    recv = torch.empty(n, dtype=torch.uint8, device=dev)
    other = 1 - rank
    ts = []
    for it in range(args.reps + 1):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops = [dist.P2POp(dist.isend, send, other), dist.P2POp(dist.irecv, recv, other)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        torch.cuda.synchronize()
        if it:
            ts.append(time.perf_counter() - t0)
    t = torch.tensor([sorted(ts)[len(ts) // 2]], dtype=torch.float64, device=dev)   # median, then max over ranks
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"peer": args.peer, "bytes_each_way": n, "seconds": float(t.item()),
                          "GBps_each_way": n / float(t.item()) / 1e9}), flush=True)
    dist.destroy_process_group()


def copy_pairs(args, ngpu):
    import torch
    n = args.mib << 20
    out = []
    src = torch.ones(n, dtype=torch.uint8, device=0)
    for j in range(1, ngpu):
        dst = torch.empty(n, dtype=torch.uint8, device=j)
        back = torch.ones(n, dtype=torch.uint8, device=j)
        dst0 = torch.empty(n, dtype=torch.uint8, device=0)
        one, both = [], []
        for it in range(args.reps + 1):
            torch.cuda.synchronize(0); torch.cuda.synchronize(j)
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize(0); torch.cuda.synchronize(j)
            t1 = time.perf_counter()
            s0, s1 = torch.cuda.Stream(0), torch.cuda.Stream(j)
            with torch.cuda.stream(s0):
                dst.copy_(src, non_blocking=True)
            with torch.cuda.stream(s1):
                dst0.copy_(back, non_blocking=True)
            torch.cuda.synchronize(0); torch.cuda.synchronize(j)
            t2 = time.perf_counter()
            if it:
                one.append(t1 - t0)
                both.append(t2 - t1)
        med = lambda xs: sorted(xs)[len(xs) // 2]
        out.append({"pair": [0, j], "copy_GBps_one_way": n / med(one) / 1e9,
                    "copy_GBps_each_way_bidirectional": n / med(both) / 1e9})
        del dst, back, dst0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--rccl-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--peer", type=int, default=1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.rccl_child:
        return rccl_pair(args)
    import torch
    ngpu = torch.cuda.device_count()   # counts without initialising the GPU on this image
    if ngpu < 2:
        print(json.dumps({"p2p_probe": "skipped", "reason": f"{ngpu} visible GPU(s): no xGMI link to measure"}))
        return 0
    rccl = []
    for j in range(1, ngpu):   # RCCL pairs first, as fresh processes (before this one initialises a GPU)
        port = 29700 + j
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rccl-child", "--peer", str(j),
                                   "--mib", str(args.mib), "--reps", str(args.reps)],
                                  env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                                           MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)),
                                  stdout=subprocess.PIPE, text=True) for r in range(2)]
        outs = [p.communicate(timeout=300)[0] for p in procs]
        if any(p.returncode for p in procs):
            sys.exit(f"p2p_probe: RCCL pair (0, {j}) failed")
        rccl.append(json.loads([x for x in outs[0].splitlines() if x.startswith("{")][-1]))
    copies = copy_pairs(args, ngpu)
    rates = sorted(r["GBps_each_way"] for r in rccl)
    rec = {"p2p_probe": "xGMI pairs (0, j)", "gpus": ngpu, "mib": args.mib, "rccl": rccl, "copy": copies,
           "link_GBps": rates[len(rates) // 2]}
    print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rec, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
