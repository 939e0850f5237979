"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch).

FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts 64 B per
TCC_EA0_RDREQ, i.e. half the bytes of 128-B (wide streaming) requests
(MI355X_MICROARCH.md, HBM): both the raw value and x2 are printed."""
import collections
import csv
import json
import sys


def short(name):
    n = name.replace("void ", "").replace("ks::(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        if "ks::" not in r["Kernel_Name"]:
            continue
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(paths):
    out = {}
    for p in paths:
        for k, cs in load(p).items():
            for c, vals in cs.items():
                out.setdefault(k, {})[c] = sum(vals) / len(vals)
                out[k]["dispatches"] = len(vals)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
