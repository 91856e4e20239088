"""profiles/rNN_point_mlp_traffic.json from a tools/pmc_profile.sh summary: the neighbour-MLP kernel's
HBM bytes (FETCH_SIZE / WRITE_SIZE passes, gfx950 read correction) and issue counters, per frame.
With early ray termination the kernel runs once per pass (ERT_PASSES launches per frame, of
different sizes): per-frame values are the per-launch averages times the launches per frame, next
to the per-frame F_alg the bench divides by the summed pass times.

    python tools/mlp_traffic.py gpurun_out/pmc/summary.txt out.json "round-5 final state" [launches_per_frame]
"""
import json
import sys


def main(summary, out, note, per_frame=9):
    d = json.load(open(summary))
    name = next(k for k in d if "k_point_mlp_h4_listed" in k or "k_point_mlp_h4<false, false, true>" in k
                or "k_point_mlp_h4<false, false>" in k)
    e = d[name]
    listed = "listed" in name or "true>" in name   # one launch per early-ray-termination pass
    per_frame = int(per_frame) if listed else 1
    res = {
        "kernel": name,
        "launches_per_frame": per_frame,
        "bytes_per_launch": e.get("hbm_bytes_per_launch", 0.0) * per_frame,
        "bytes_per_launch_note": "per frame: the average launch's (2*FETCH_SIZE + WRITE_SIZE)*1024 times the "
                                 "launches per frame (the bench's roofline is per frame: all passes' rows over "
                                 "all passes' time)",
        "avg_ms": e["avg_ms"] * per_frame,
        "FETCH_SIZE_KB": e.get("FETCH_SIZE"), "WRITE_SIZE_KB": e.get("WRITE_SIZE"),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py --in-flight 1 "
                  "(tools/pmc_profile.sh); bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (MI355X_MICROARCH.md gfx950 "
                  "read correction); " + note,
    }
    if e.get("SQ_INSTS_MFMA"):
        res["valu_per_mfma"] = e.get("SQ_INSTS_VALU", 0) / e["SQ_INSTS_MFMA"]
        res["valu_non_mfma_per_mfma"] = (e.get("SQ_INSTS_VALU", 0) - e["SQ_INSTS_MFMA"]) / e["SQ_INSTS_MFMA"]
    for k_out, k_in in (("mfma_busy_frac", "mfma_busy_frac"), ("eff_clock_GHz", "eff_clock_GHz")):
        if k_in in e:
            res[k_out] = e[k_in]
    if e.get("SQ_WAVE_CYCLES"):
        res["sq_wait_any_frac"] = e.get("SQ_WAIT_ANY", 0) / e["SQ_WAVE_CYCLES"]
        res["sq_wait_inst_any_frac"] = e.get("SQ_WAIT_INST_ANY", 0) / e["SQ_WAVE_CYCLES"]
    if e.get("SQ_INSTS_LDS"):
        res["lds_bank_conflict_per_lds_inst"] = e.get("SQ_LDS_BANK_CONFLICT", 0) / e["SQ_INSTS_LDS"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
