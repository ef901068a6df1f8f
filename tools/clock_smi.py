"""Poll amdsmi's gpu_metrics clocks while a command runs (calibration of the in-kernel clock probe).

python tools/clock_smi.py <out.jsonl> -- <cmd...>
Writes one JSON object per poll (t, every *clk* field of gpu_metrics) and the command's own stdout.
"""
import json
import subprocess
import sys
import time

out_path = sys.argv[1]
cmd = sys.argv[sys.argv.index("--") + 1:]
try:
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
except Exception as e:  # noqa: BLE001 -- report, run the command anyway
    print("amdsmi unavailable:", repr(e))
    h = None

p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
t0 = time.time()
with open(out_path, "w") as f:
    while p.poll() is None:
        if h is not None:
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(h)
                rec = {"t": round(time.time() - t0, 4)}
                for k, v in m.items():
                    if "clk" in k.lower() or "power" in k.lower() or "activity" in k.lower():
                        rec[k] = v
                f.write(json.dumps(rec, default=str) + "\n")
            except Exception as e:  # noqa: BLE001
                f.write(json.dumps({"t": time.time() - t0, "err": repr(e)}) + "\n")
                h = None
        time.sleep(0.005)
print(p.stdout.read())
sys.exit(p.returncode)
