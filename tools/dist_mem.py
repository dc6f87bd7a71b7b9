#!/usr/bin/env python3
"""Per-rank device memory of the sharded Stark::prove (sg_dist_stark_prove) at world G (VERDICT r05
"Next round" 3; stark/stark.rs:276-562): G ranks on this one GPU over the host transport (gloo), the
bench's Rescue-Prime statement with a trace of 2^L rows.  Every rank proves twice (the first proof
builds the context's public tables); its pool high-water mark is reset before the second, so

  peak      = the buffer pool's high-water mark of one steady-state sharded proof on this rank
              (its codeword shards, retained FRI / forest trees, gathered quotients, scratch)
  resident  = device bytes this rank's context holds across proofs besides its pool (twiddle plans,
              domain / AIR tables incl. the replicated trace-domain tables), measured by hipMemGetInfo
              around closing the context minus the pool's bytes, one rank at a time (barriers keep
              the other ranks' memory fixed meanwhile)
  total     = peak + resident: the device memory one rank needs

Each rank's context is its own, so these are exactly what a rank on its own GPU would hold.
usage: dist_mem.py L G [G ...]      prints one JSON line per (L, G), rank 0's and the max over ranks
"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zk-stark-tutor_amd")]


def _worker(rank, world, port, L, out_path):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from starkgpu import dist as D
    sg = bench.sg
    dev = torch.device("cuda", 0)
    ctx = sg.Context(0)
    nd = D.NativeDist(ctx, transport="host")
    wl = bench.ProveWorkload(0, dev, ctx, L)

    def prove():
        ps = sg.IndependentProofStream()
        wl.stark.prove_dev(wl.trace.data_ptr(), wl.rows, wl.air, wl.boundary, ps, wl.trace_rand.data_ptr(),
                           wl.rcoef.data_ptr(), wl.nrc, dist=nd)
        return ps.digest()

    first = prove()
    torch.cuda.synchronize(dev)
    ctx.memory(reset_peak=True)
    second = prove()
    torch.cuda.synchronize(dev)
    assert first == second
    peak = ctx.memory()["peak"]
    digest = __import__("hashlib").sha256(second).hexdigest()
    nd.close()
    resident = None
    for r in range(world):
        dist.barrier()
        if r == rank:
            torch.cuda.synchronize(dev)
            m = ctx.memory()  # the pool's free cache holds the peak's buffers (counted in `peak`)
            free_before, _ = torch.cuda.mem_get_info(dev)
            del wl.stark, wl.air, wl.rp  # library objects on this context (the trace tensors stay: caller memory)
            ctx.close()  # frees the pool and every table the context keeps
            torch.cuda.synchronize(dev)
            free_after, _ = torch.cuda.mem_get_info(dev)
            resident = free_after - free_before - m["pooled"] - m["live"]
        dist.barrier()
    rows = [None] * world
    dist.all_gather_object(rows, {"rank": rank, "peak": peak, "resident": resident, "digest": digest,
                                  "fri_domain": wl.fri_len})
    if rank == 0:
        tot = [r["peak"] + r["resident"] for r in rows]
        line = {"log_trace": L, "world": world, "fri_domain": rows[0]["fri_domain"],
                "fri_per_rank": rows[0]["fri_domain"] // world,
                "rank0": {"peak": rows[0]["peak"], "resident": rows[0]["resident"], "total": tot[0]},
                "max_total": max(tot), "max_peak": max(r["peak"] for r in rows),
                "max_resident": max(r["resident"] for r in rows),
                "bytes_per_fri_element_per_rank": round(max(tot) / (rows[0]["fri_domain"] // world), 1),
                "proof_bytes_equal_across_ranks": len({r["digest"] for r in rows}) == 1}
        print(json.dumps(line), flush=True)
        with open(out_path, "a") as f:
            f.write(json.dumps(line) + "\n")
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    L = int(sys.argv[1])
    out = os.environ.get("SG_DIST_MEM_OUT", os.path.join(ROOT, "gpurun_out", "dist_mem.jsonl"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    for G in [int(g) for g in sys.argv[2:]]:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.spawn(_worker, args=(G, port, L, out), nprocs=G, join=True)


if __name__ == "__main__":
    main()
