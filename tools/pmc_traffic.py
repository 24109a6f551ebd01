"""Per-launch HBM traffic of each bench phase from tools/profile.sh PMC passes -> profiles/pmc_traffic.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (both counters in KB; FETCH_SIZE x 2 is the gfx950
correction of MI355X_MICROARCH.md's rocprofv3 section).  Only phases that are a single kernel are mapped.
usage: python tools/pmc_traffic.py PROFILE_DIR N W H
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import avg, load_counters  # noqa: E402

# bench phase -> its kernels (names as pmc_summary._short gives them; phases whose kernels are also launched by the
# gated phase-2 path under the same name are left out)
PHASE_KERNEL = {
    "preprocess": ["k_preprocess"], "emit": ["k_bin_count<1>", "k_bin_emit<1>"], "render_fwd": ["k_render_fwd<1>"],
    "render_bwd": ["k_bwd_prologue", "k_render_bwd"], "gauss_bwd": ["k_gauss_sum", "k_gauss_live"],
}


def main(root, n, W, H):
    acc = load_counters(root)
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                            "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    key = f"{n}x{W}x{H}"
    ent = {}
    for phase, kerns in PHASE_KERNEL.items():
        cs = [acc.get(k) for k in kerns]
        if not all(c and "FETCH_SIZE" in c for c in cs):
            continue
        ent[phase] = sum((2.0 * avg(c["FETCH_SIZE"]) + avg(c.get("WRITE_SIZE", [0.0]))) * 1024.0 for c in cs)
    d[key] = ent
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(key, {k: round(v / 1e6, 1) for k, v in ent.items()}, "MB")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
