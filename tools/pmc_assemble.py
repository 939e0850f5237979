"""profiles/pmc_summary.json from the rocprofv3 --pmc passes of
tools/gpu_pmc.sh (one counter group per run, `bench.py --steps 1 --warmup 0
--no-cpu`): per kernel the average FETCH_SIZE / WRITE_SIZE (KB) per dispatch
and the dispatch count, tagged with the library build id and the workload
bench.py compares before using them (bench.py pmc_traffic).

  python tools/pmc_assemble.py BENCH_JSON OUT_JSON PASS_CSV...
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main(bench_json, out_json, *csvs):
    b = json.load(open(bench_json))
    cfg = b["config"]
    kernels = {}
    for p in csvs:
        for name, cs in load(p).items():
            for c, vals in cs.items():
                kernels.setdefault(name, {})[c] = sum(vals) / len(vals)
                kernels[name]["dispatches"] = len(vals)
    n_bases = int(cfg["genome_bp"])
    p1 = cfg.get("pass1_kernel", "k_pass1p")
    out = {
        "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, tools/gpu_pmc.sh) of "
                "`python bench.py --steps 1 --warmup 0 --no-cpu`; values in KB per dispatch (raw counters: "
                "FETCH_SIZE = TCC_EA0_RDREQ x 64 B, so 128-B streaming reads count half, MI355X_MICROARCH.md); "
                "the scan's pass 1 is two dispatches per step (the two parts of the runs).",
        "build_id": cfg["build_id"],
        "workload": {"k": cfg["k"], "score": cfg["score"], "scale": 1.0, "ncontigs": 24, "expand": True,
                     "trlr": False, "mode": cfg["mode"], "world": 1},
        # scan calls in the profiled run: its steps + warmup, plus the visits
        # line's warm call and 3 timed calls (the same scan)
        "steps": int(b["steps"]) + int(b["warmup"]) + (4 if b.get("visits_path") else 0),
        # packed bases (total / 4 bytes per step) are the only 16-B streaming read of the pass-1 kernel
        "streaming_read_bytes_per_step": {p1: n_bases / 4.0},
        "kernels": kernels,
    }
    json.dump(out, open(out_json, "w"), indent=1)
    kp = {k: v for k, v in kernels.items() if k.startswith(p1)}
    print(json.dumps(kp, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
