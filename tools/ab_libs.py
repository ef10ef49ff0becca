"""Interleaved A/B of library builds on the GPU box: for each round, each
library (TPST_LIB_PATH) runs the headline MSM bench (bench.py, MSM leg only)
and the Fq29 microbenchmarks in a child process.  JSON lines.

    python tools/ab_libs.py ROUNDS label=path/to/libtpst.so ...
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(label, path):
    env = dict(os.environ, TPST_LIB_PATH=os.path.join(ROOT, path))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-pst", "--no-sharded",
                        "--no-r1cs", "--no-groth16", "--steps", "20", "--warmup", "3"], capture_output=True, text=True,
                       env=env, timeout=300)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[-1]) if line else {"error": r.stderr[-2000:]}
    m = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mb_fq29.py")], capture_output=True, text=True,
                       env=env, timeout=300)
    mb = [json.loads(x) for x in m.stdout.splitlines() if x.startswith("{")]
    return {"label": label, "value": d.get("value"), "ms_per_step": d.get("ms_per_step"),
            "latency_ms": d.get("latency_ms_single_call"),
            "stages": d.get("stages_ms_per_step"), "mb": {x["op"]: [x["chip_G_per_s"], x["lone_wave_us"]] for x in mb}}


def main():
    rounds = int(sys.argv[1])
    libs = [a.split("=", 1) for a in sys.argv[2:]]
    for _ in range(rounds):
        for label, path in libs:
            print(json.dumps(run(label, path)), flush=True)


if __name__ == "__main__":
    main()
