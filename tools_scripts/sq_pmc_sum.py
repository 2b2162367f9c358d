"""Sum rocprofv3 --pmc counter rows per kernel (the bench process's largest
counter_collection.csv) and print per-kernel shares of wave cycles."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
f = max(fs, key=os.path.getsize)
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
for k, c in rows[:12]:
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:40s} disp {len(disp[k]):5d} waves {c.get('SQ_WAVES',0):12.0f} "
          f"valu_insts {c.get('SQ_INSTS_VALU',0):14.0f} salu {c.get('SQ_INSTS_SALU',0):12.0f} "
          f"active_valu {c.get('SQ_ACTIVE_INST_VALU',0)/w:.3f} active_any {c.get('SQ_ACTIVE_INST_ANY',0)/w:.3f} "
          f"wait_any {c.get('SQ_WAIT_ANY',0)/w:.3f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/w:.3f}")
