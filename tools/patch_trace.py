"""Summarise the DEEP launches of a patch-latency kernel trace (rocprofv3 --kernel-trace csv):
launch durations, gaps between launches, the job-array copies, and how busy the GPU was.

python tools/patch_trace.py profiles/r06_patch/kernel_trace_16.csv profiles/r06_patch/patch_16.json
"""
import csv
import json
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
deep = [r for r in rows if "deep_kernel" in r["Kernel_Name"]]
cp = [r for r in rows if "copyBuffer" in r["Kernel_Name"]]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in deep]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e6 for a, b in zip(deep, deep[1:])]
span = (int(deep[-1]["End_Timestamp"]) - int(deep[0]["Start_Timestamp"])) / 1e6
print(f"DEEP launches {len(dur)}: median {st.median(dur):.3f} ms (min {min(dur):.3f}, max {max(dur):.3f}); "
      f"gaps median {st.median(gaps) * 1e3:.1f} us, max {max(gaps):.3f} ms; busy {sum(dur) / span:.4f} of {span:.1f} ms")
print(f"job-array copies {len(cp)}: median "
      f"{st.median((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in cp):.1f} us")
if len(sys.argv) > 2:
    h = json.load(open(sys.argv[2]))
    p50 = h["patch_group_ms"]["p50"]
    launch = st.median(dur)
    per = h["jobs"] / h["uploads"]
    print(f"PATCH p50 {p50:.2f} ms = {per:.0f} own launches x {launch:.3f} ms + {p50 - per * launch:.2f} ms "
          f"({(p50 - per * launch) / launch:.2f} launches) waiting; {h['jobs'] / h['launches']:.1f} jobs per launch")
