"""Summarise k_env0 sweep runs: python scripts/envsum.py gpurun_out/<tag>_c3_*/"""
import csv, json, os, sys
for d in sys.argv[1:]:
    d = d.rstrip("/")
    rows = {r["Name"]: r for r in csv.DictReader(open(d + "/run_kernel_stats.csv"))}
    env = [float(r["AverageNs"]) / 1e3 for k, r in rows.items() if "k_env0" in k]
    fix = sum(float(r["AverageNs"]) / 1e3 * int(r["Calls"]) / 13 for k, r in rows.items() if "k_envfix" in k)
    ms = ef = par = None
    if os.path.exists(d + ".log"):
        ls = [l for l in open(d + ".log") if l.startswith('{"metric"')]
        if ls:
            j = json.loads(ls[-1]); ms = j["ms_per_step"]; ef = j.get("env_fixup"); par = j.get("plan")
    print(os.path.basename(d), "env0 %.1f us" % env[0], "fix/step %.1f us" % fix, "ms/step", ms, ef)
