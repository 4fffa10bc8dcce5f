"""Summarise rocprofv3 PMC counter CSVs per kernel (averaged per dispatch).

    python scripts/pmc_summary.py gpurun_out/pmc_TAG_sq/run_counter_collection.csv [...]

SQ_* wave/cycle counters are in quad-cycles (MI355X_MICROARCH.md); the derived
columns are VALU = ACTIVE_INST_VALU / BUSY-per-SIMD proxy, wait fractions of
WAVE_CYCLES.
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:amx::)?([A-Za-z0-9_]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for fn in sys.argv[1:]:
        for r in csv.DictReader(open(fn)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((fn, r["Dispatch_Id"]))
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        n = max(1, len(disp[k]) // max(1, len(sys.argv) - 1))
        row = {c: x / n for c, x in v.items()}
        wc = row.get("SQ_WAVE_CYCLES", 0)
        extra = ""
        if wc:
            extra = " waitany %.2f waitinst %.2f active %.2f valu/active %.2f" % (
                row.get("SQ_WAIT_ANY", 0) / wc, row.get("SQ_WAIT_INST_ANY", 0) / wc,
                row.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                row.get("SQ_ACTIVE_INST_VALU", 0) / max(1, row.get("SQ_ACTIVE_INST_ANY", 1)))
        print("%-32s %s%s" % (k[:32], " ".join("%s=%.3g" % (c.replace("SQ_", ""), x) for c, x in sorted(row.items())), extra))


if __name__ == "__main__":
    main()
