"""Summarise tools/ab_inproc.py outputs: variant, min / median ms, best-step phases."""
import json
import sys

for f in sys.argv[1:]:
    print("==", f)
    for line in open(f):
        i = line.find("{")
        if 0 <= i < 30:
            try:
                d = json.loads(line[i:])
            except ValueError:
                continue
            ph = " ".join(f"{k[3:]}={v}" for k, v in d.get("best_phases", {}).items())
            print(f"  {line[:i].strip():10s} min {d.get('min_ms')} med {d.get('median_ms')}  {ph}")
        elif "differ" in line or "mismatch" in line.lower():
            print("  " + line.rstrip())
