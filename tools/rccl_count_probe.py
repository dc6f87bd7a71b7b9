#!/usr/bin/env python3
"""Probe of the round-4 RCCL defect (VERDICT r05 "Next round" 5): a single 2 GiB all-to-all on a
one-rank communicator returned wrong data when issued as ncclUint8 (count 2^31).  This issues the
same exchange through torch.distributed (backend "nccl" = RCCL) with the element type varied, so
the count varies at fixed bytes: uint8 (2^31 elements), int32 (2^29), int64 (2^28); and below the
boundary (2^31 - 256 bytes as uint8).  Each line: dtype, count, bytes, and whether the received
buffer equals the sent one (world 1: all-to-all and all-gather are copies).

usage: rccl_count_probe.py [log2_bytes]   (default 31)
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
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
