#!/usr/bin/env python3
"""Run a command and sample the GPU's clocks, power and temperature beside it.

Used to attribute the drop from the bench's 20-step window rate to the rate
sustained over the ~4-minute time-to-converge run: the
samples show whether the shader clock falls as the run goes on.

  python tools/clock_sampler.py --every 10 --out gpurun_out/x/clocks.jsonl -- python bench.py ...

The command runs as a child process (never exec'd into); this script exits
with the child's exit code.  Each sample is one JSON line: seconds since the
start and `rocm-smi -c -P -t -u --json` for the devices (raw strings; the
summary keeps the sclk / power / temperature fields it finds).
"""
import argparse
import json
import re
import subprocess
import sys
import time


def sample():
    try:
        r = subprocess.run(["rocm-smi", "-c", "-P", "-t", "-u", "--json"], capture_output=True, text=True, timeout=20)
        return json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else {"error": r.stderr[-300:]}
    except (OSError, subprocess.TimeoutExpired, json.JSONDecodeError) as e:
        return {"error": str(e)}


def pick(card):
    """The fields that matter for a clock-down, from one card's rocm-smi record."""
    out = {}
    for k, v in card.items():
        kl = k.lower()
        if "sclk" in kl or "power" in kl or ("temperature" in kl and ("junction" in kl or "edge" in kl)) or "gpu use" in kl:
            m = re.search(r"[-+]?\d+(\.\d+)?", str(v))
            out[k] = float(m.group()) if m else v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=float, default=10.0)
    ap.add_argument("--out", required=True)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("no command after --")
    t0 = time.time()
    child = subprocess.Popen(cmd)
    with open(a.out, "w") as f:
        while True:
            s = sample()
            rec = {"t": round(time.time() - t0, 1)}
            if isinstance(s, dict) and "error" not in s:
                rec["cards"] = {c: pick(v) for c, v in s.items() if isinstance(v, dict)}
            else:
                rec["error"] = s.get("error") if isinstance(s, dict) else str(s)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            try:
                child.wait(timeout=a.every)
                break
            except subprocess.TimeoutExpired:
                pass
    sys.exit(child.returncode)


if __name__ == "__main__":
    main()
