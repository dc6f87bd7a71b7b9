#!/usr/bin/env python3
"""Probe of the round-4 RCCL defect (VERDICT r05 "Next round" 5): a single 2 GiB all-to-all on a
one-rank communicator returned wrong data when issued as ncclUint8 (count 2^31).  This issues the
same exchange through torch.distributed (backend "nccl" = RCCL) with the element type varied, so
the count varies at fixed bytes: uint8 (2^31 elements), int32 (2^29), int64 (2^28); and below the
boundary (2^31 - 256 bytes as uint8).  Each line: dtype, count, bytes, and whether the received
buffer equals the sent one (world 1: all-to-all and all-gather are copies).

usage: rccl_count_probe.py [log2_bytes]   (default 31)
       rccl_count_probe.py sweep           all-to-all (int64) at sizes between 1 GiB and 2 GiB
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def sweep():
    """all_to_all_single, int64 elements, world 1: the largest per-call size that stays exact."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29534")
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    top = 1 << 31
    src = torch.randint(0, 256, (top,), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    gib = 1 << 30
    for nb in (gib - 256, gib, gib + 256, gib + (1 << 20), gib + (1 << 23), gib + (1 << 24), gib + (1 << 28),
               gib + (1 << 29), top - (1 << 28), top - 256, top):
        s, d = src[:nb].view(torch.int64), dst[:nb].view(torch.int64)
        d.fill_(0)
        torch.cuda.synchronize()
        dist.all_to_all_single(d, s)
        torch.cuda.synchronize()
        eq = d.view(torch.uint8) == s.view(torch.uint8)
        ok = bool(eq.all().item())
        first_bad = -1 if ok else int(torch.argmin(eq.to(torch.uint8)).item())
        print("all_to_all int64 bytes %11d (%.6f GiB)  equal %s  first wrong byte %d" % (nb, nb / gib, ok, first_bad),
              flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        return sweep()
    logb = int(sys.argv[1]) if len(sys.argv) > 1 else 31
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    nbytes = 1 << logb
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g)
    dst = torch.empty_like(src)
    cases = [(torch.uint8, nbytes), (torch.int32, nbytes), (torch.int64, nbytes), (torch.uint8, nbytes - 256)]
    for dtype, nb in cases:
        esz = torch.tensor([], dtype=dtype).element_size()
        s = src[:nb].view(dtype)
        for op in ("all_to_all_single", "all_gather_into_tensor"):
            d = dst[:nb].view(dtype)
            d.fill_(0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if op == "all_to_all_single":
                dist.all_to_all_single(d, s)
            else:
                dist.all_gather_into_tensor(d, s)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok = bool(torch.equal(d.view(torch.uint8), s.view(torch.uint8)))
            bad = int((d.view(torch.uint8) != s.view(torch.uint8)).sum().item()) if not ok else 0
            print("%-24s %-12s count %11d (2^%.2f)  bytes %11d  equal %s  mismatched bytes %d  %.1f ms"
                  % (op, str(dtype).replace("torch.", ""), nb // esz, (nb // esz).bit_length() - 1 +
                     ((nb // esz) / (1 << ((nb // esz).bit_length() - 1)) - 1), nb, ok, bad, dt * 1e3), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
