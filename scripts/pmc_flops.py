"""FLOPs per kernel launch from one rocprofv3 PMC pass over the VALU instruction counters.

    python scripts/pmc_flops.py COUNTER_CSV OUT_JSON

SQ_INSTS_VALU_* count wave instructions (summed over the SEs by rocprofv3); a wave
instruction is 64 lanes, an FMA 2 FLOPs (the counter_defs.yaml FLOP expressions).
Lanes masked off still count: these are issued FLOPs.  TRANS (rcp, sqrt, exp, log)
count 1 each.  Averaged over every dispatch of a kernel."""
import collections
import csv
import json
import re
import sys

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64")
F32 = ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32")


def short(name):
    m = re.match(r"(?:void )?(?:amx::)?([A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = short(r["Kernel_Name"])
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = {"source": "rocprofv3 --pmc " + " ".join(F64 + F32) + " (one pass)",
           "flops": "64 lanes x (2 FMA + ADD + MUL + TRANS) per wave instruction, issued",
           "kernels": {}}
    for k, c in tot.items():
        n = max(1, len(disp[k]))
        f64 = 64.0 * (2 * c[F64[0]] + c[F64[1]] + c[F64[2]] + c[F64[3]]) / n
        f32 = 64.0 * (2 * c[F32[0]] + c[F32[1]] + c[F32[2]] + c[F32[3]]) / n
        out["kernels"][k] = {"fp64_flops": round(f64), "fp32_flops": round(f32), "launches": n}
    json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["fp64_flops"]):
        print("%-24s fp64 %12.3f GFLOP  fp32 %12.3f GFLOP  (%d launches)" %
              (k, v["fp64_flops"] / 1e9, v["fp32_flops"] / 1e9, v["launches"]))


if __name__ == "__main__":
    main()
