#!/usr/bin/env python3
"""Write `rocprofv3 --list-avail` (the PMC counters this GPU exposes) to a file.

  python tools/probes/list_counters.py OUT.txt
"""
import subprocess
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "counters.txt"
r = subprocess.run(["rocprofv3", "--list-avail"], capture_output=True, text=True, timeout=120)
with open(out, "w") as f:
    f.write(r.stdout)
    f.write(r.stderr)
print("rc", r.returncode, "lines", (r.stdout + r.stderr).count("\n"))
sys.exit(r.returncode)
