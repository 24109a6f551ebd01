"""Per-launch HBM traffic and VALU figures of each bench phase from tools/profile.sh's rocprofv3 passes
-> profiles/pmc_traffic.json (read by bench.py for roofline.traffic and roofline.valu).

Per phase (the sum over its kernels, each averaged per dispatch):
  hbm_bytes   (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (both counters in KB; FETCH_SIZE x 2 is the gfx950 correction of
              MI355X_MICROARCH.md's rocprofv3 section)
  valu_insts  SQ_INSTS_VALU (wave-instructions, summed over the launch's waves)
  valu_busy   SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (kernel-trace duration in cycles x 1024 SIMDs)
  us          kernel-trace duration
Kernels are matched by name prefix (pmc_summary._short names); phase-2 kernels launched under the same names by the
gated phase-2 path are the '<2' template instances and are not matched.
usage: python tools/pmc_traffic.py PROFILE_DIR N W H [SUFFIX]   (key "{N}x{W}x{H}{SUFFIX}", e.g. SUFFIX -sparse)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import CLOCK_GHZ, SIMDS, avg, load_counters, load_durations  # noqa: E402

PHASE_KERNELS = {
    "preprocess": ["k_preprocess"],
    "emit": ["k_bin_count<1", "k_bin_offsets", "k_bin_emit<1"],
    "render_fwd": ["k_render_fwd<1"],
    "render_bwd": ["k_bwd_prologue", "k_render_bwd"],
    "gauss_bwd": ["k_gauss_sum", "k_gauss_live"],
}


def main(root, n, W, H, suffix=""):
    acc = load_counters(root)
    dur = load_durations(root)
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                            "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    key = f"{n}x{W}x{H}{suffix}"
    ent = {}
    for phase, prefixes in PHASE_KERNELS.items():
        ks = sorted({k for k in set(acc) | set(dur) for p in prefixes if k.startswith(p)})
        if not ks:
            continue
        e = {"kernels": ks, "us": sum(avg(dur.get(k, [])) for k in ks)}
        cs = [acc.get(k, {}) for k in ks]
        if all("FETCH_SIZE" in c for c in cs):
            e["hbm_bytes"] = sum((2.0 * avg(c["FETCH_SIZE"]) + avg(c.get("WRITE_SIZE", [0.0]))) * 1024.0 for c in cs)
        if all("SQ_INSTS_VALU" in c for c in cs):
            e["valu_insts"] = sum(avg(c["SQ_INSTS_VALU"]) for c in cs)
        if all("SQ_ACTIVE_INST_VALU" in c for c in cs) and e["us"] > 0:
            e["valu_busy"] = round(sum(avg(c["SQ_ACTIVE_INST_VALU"]) for c in cs) * 4.0
                                   / (e["us"] * 1e-6 * CLOCK_GHZ * 1e9 * SIMDS), 4)
        ent[phase] = e
    d[key] = ent
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(ent, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else "")
