"""Instruction mix of an inner loop in compiled gfx950 ISA (hipcc --cuda-device-only -S): counts the instructions
between two labels of a kernel by class -- the attribution table of DESIGN.md §8.
python tools/isa_mix.py FILE.s FUNCTION START_LABEL END_LABEL"""
import re
import sys
from collections import Counter

CLASSES = [
    ("transcendental (v_exp/v_rcp)", r"^v_(exp|rcp|rsq|log|sqrt)_f32"),
    ("packed fp32 (v_pk_*)", r"^v_pk_"),
    ("fma / mul / add / sub (scalar fp32)", r"^v_(fma|fmac|mul|add|sub|subrev|mad)_f32(?!_dpp)"),
    ("DPP add / move (cross-lane)", r"_dpp$|^v_mov_b32_dpp|^v_add_f32_dpp"),
    ("permlane swap (cross-lane)", r"^v_permlane"),
    ("select (v_cndmask)", r"^v_cndmask"),
    ("compare (v_cmp*)", r"^v_cmp"),
    ("min / max", r"^v_(min|max)_f32"),
    ("move / readlane / other VALU", r"^v_"),
    ("LDS (ds_*)", r"^ds_"),
    ("global memory", r"^(global|buffer|flat)_"),
    ("SALU / branch / wait (s_*)", r"^s_"),
]


def main():
    path, fn, start, end = sys.argv[1:5]
    lines = open(path).read().splitlines()
    i0 = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    a = next(i for i in range(i0, len(lines)) if lines[i].startswith(start + ":"))
    b = next(i for i in range(a + 1, len(lines)) if lines[i].startswith(end + ":") or lines[i].startswith(end))
    cnt, total = Counter(), 0
    for l in lines[a:b]:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        total += 1
        for name, rx in CLASSES:
            if re.search(rx, op):
                cnt[name] += 1
                break
        else:
            cnt["other"] += 1
    valu = sum(v for k, v in cnt.items() if not k.startswith(("LDS", "global", "SALU")))
    print(f"{fn} [{start}, {end}): {total} instructions, {valu} VALU")
    for name, _ in CLASSES + [("other", "")]:
        if cnt[name]:
            print(f"  {name:40s} {cnt[name]:4d}")


if __name__ == "__main__":
    main()
