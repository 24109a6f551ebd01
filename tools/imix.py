"""Instruction mix of the render kernels from the tools/pmc_imix.txt passes of tools/profile.sh (rocprofv3 --pmc).

usage: python tools/imix.py OUTDIR [KERNEL ...]     (default kernels: k_render_bwd, k_render_fwd<1, false>)

Per kernel, averaged per dispatch: each counter's value, per wave (SQ_WAVES), and the cycle-type counters (quad-cycles,
summed over waves: x4 / waves) per wave.  The per-splat figures divide by the replay / compositing steps the bench's
view statistics give (--steps-per-wave).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load_counters, load_durations  # noqa: E402

QUAD = ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
        "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("kernels", nargs="*", default=["k_render_bwd", "k_render_fwd<1, false>"])
    a = ap.parse_args()
    acc = load_counters(a.out)
    dur = load_durations(a.out)
    for want in a.kernels:
        names = [k for k in acc if want in k]
        if not names:
            print(f"{want}: no counters")
            continue
        k = names[0]
        c = {n: sum(v) / len(v) for n, v in acc[k].items() if v}
        waves = c.get("SQ_WAVES", 0.0)
        d = dur.get(k) or next((v for n, v in dur.items() if want in n), None)
        us = sum(d) / len(d) if d else float("nan")
        print(f"== {k}  ({us:.1f} us per dispatch, {waves:.0f} waves)")
        for n in sorted(c):
            v = c[n]
            per = v / waves if waves else float("nan")
            q = "  (x4 cycles/wave: %.0f)" % (4 * per) if n in QUAD else ""
            print(f"  {n:34s} {v:16.0f}  per wave {per:12.1f}{q}")
        if waves and "SQ_INSTS_VALU" in c:
            valu = c["SQ_INSTS_VALU"]
            typed = sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                                                  "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
                                                  "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_INT32"))
            print(f"  VALU not in the typed counters (moves, compares, selects, DPP/permlane, packed?): "
                  f"{(valu - typed) / waves:.1f} per wave ({100 * (valu - typed) / valu:.1f}%)")


if __name__ == "__main__":
    main()
