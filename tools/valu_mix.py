#!/usr/bin/env python3
"""Static VALU mix roof of the hot kernels from the gfx950 listing (make -C zk-stark-tutor_amd asm).

Per-op issue rates measured on MI355X (tools/microbench_int.hip,
profiles/r01_microbench_int_v2.txt, wave-instr per CU per clock with two waves per SIMD):
plain 32-bit add/sub/xor/and/or/bitop3/shift-right/mov issue at ~1.65 (~2.4 clk per
wave64 instruction per SIMD -- the guide's 2-clk SIMD-32 rate, MI355X_MICROARCH.md:54);
everything else the hot loops use (32-bit multiplies and mads, add/sub with carry,
alignbit/alignbyte/perm, 64-bit shifts and lshl_add, 3-input ops, DPP/SDWA) issues at
~0.9 (~4.4 clk).  The mix roof of a kernel = 1024 SIMDs x clock / (weighted clk per
instruction) over its static VALU mix (the leaf kernel is straight-line code, so the
static mix is its dynamic mix; for loops it is an approximation).

usage: valu_mix.py LISTING.s OUT_JSON
"""
import json
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from asm_mix import kernels  # noqa: E402

FULL_CLK, HALF_CLK = 4 / 1.65, 4 / 0.90
FULL = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|xor_b32|and_b32|or_b32|not_b32|bitop3_b32|bitop3_b16|"
                  r"lshrrev_b32|ashrrev_i32|mov_b32|cndmask_b32|max_u32|min_u32)(_e32|_e64)?$")
KERNELS = {"merkle_leaves": "k_merkle_leaf_pairsILi512ELb0E", "merkle_fold_leaves": "k_merkle_leaf_pairsILi512ELb1E",
           "merkle_nodes": "k_merkle_levelsILb0ELi256ELb0E", "ntt_pass": "k_ntt_pass_rrILi11E",
           "ntt_first": "k_ntt_firstILi11E"}


def mix(body):
    full = half = 0
    for line in body:
        t = line.strip()
        if not t.startswith("v_"):
            continue
        op = t.split()[0]
        if "_dpp" in t or "sdwa" in t or op.endswith("_sdwa"):
            half += 1
        elif FULL.match(op) and not op.startswith("v_lshlrev_b32_e64"):
            full += 1
        else:
            half += 1
    return full, half


def main():
    listing, out = sys.argv[1], sys.argv[2]
    res = {}
    bodies = dict(kernels(listing))
    for alias, sub in KERNELS.items():
        for name, body in bodies.items():
            if sub in name:
                f, h = mix(body)
                clk = (f * FULL_CLK + h * HALF_CLK) / (f + h)
                res[alias] = {"valu_static": f + h, "full_rate": f, "half_rate": h,
                              "half_frac": round(h / (f + h), 4), "clk_per_wave_instr_per_simd": round(clk, 3)}
                break
    json.dump({"source": "static VALU mix of zk-stark-tutor_amd/build/kernels-gfx950.s; rates from "
                         "profiles/r01_microbench_int_v2.txt (full 1.65, half 0.90 wave-instr/CU/clk)",
               "full_clk": round(FULL_CLK, 3), "half_clk": round(HALF_CLK, 3), "kernels": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
