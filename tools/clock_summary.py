"""Summarise tools/clock_probe.sh output: per kernel name, mean duration, GRBM_GUI_ACTIVE / duration
/ 8 XCDs
(the counter is summed over the 8 XCD instances: the shader clock while the kernel ran) and
SQ_VALU_MFMA_BUSY_CYCLES per GRBM cycle per CU (a relative MFMA-busy figure for A/B only)."""
import csv, glob, sys, collections

out, tag = sys.argv[1], sys.argv[2]
cc = glob.glob(f"{out}/**/*counter_collection.csv", recursive=True)
if not cc:
    sys.exit("no counter_collection.csv")
rows = list(csv.DictReader(open(cc[0])))
per = collections.defaultdict(lambda: collections.defaultdict(float))
durs = collections.defaultdict(list)
seen = set()
for r in rows:
    name = r.get("Kernel_Name", "")
    key = (r.get("Dispatch_Id"), name)
    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    if "Start_Timestamp" in r and key not in seen:
        seen.add(key)
        durs[key] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
for key, c in per.items():
    short = key[1].split("(")[0][-60:]
    a = agg[short]
    a[0] += 1
    a[1] += durs.get(key, 0.0)
    a[2] += c.get("GRBM_GUI_ACTIVE", 0.0)
    a[3] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    a[4] += c.get("SQ_BUSY_CYCLES", 0.0)
for short, (n, d, g, m, b) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:6]:
    if d <= 0:
        continue
    print(f"{tag:8s} {short:60s} n={n} avg_ms={d / n / 1e6:.3f} clk_GHz={g / d / 8:.3f} mfma_busy_rel={m / max(g, 1) / 256:.3f}")
