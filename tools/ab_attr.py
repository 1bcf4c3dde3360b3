"""Same-box interleaved A/B of bench.py with module attributes set in-process (the A/B hooks
of the package, e.g. ops.gemm_select.TN_GROUP), each run a fresh subprocess:

    python tools/ab_attr.py --rounds 2 "" "ops.gemm_select.TN_GROUP=False" "ext:gemm4_m32(0)" -- --steps 20

(an arm is a ';'-separated list of module.ATTR=value and ext:<native call>)
prints ms/step and tok/s per arm and run, then the per-arm means."""
import json
import subprocess
import sys

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def run(arm, bench_args):
    sets = []
    for kv in filter(None, arm.split(";")):
        if kv.startswith("ext:"):   # a native A/B switch, e.g. ext:gemm4_m32(0)
            sets.append(f"from distributed_pytorch_from_scratch_amd.ops import _ext; _ext.require().{kv[4:]}")
            continue
        path, val = kv.split("=")
        mod, attr = path.rsplit(".", 1)
        sets.append(f"import distributed_pytorch_from_scratch_amd.{mod} as _m; _m.{attr} = {val}")
    code = "; ".join(sets + ["import runpy, sys", f"sys.argv = ['bench.py'] + {bench_args!r}",
                             "runpy.run_path('bench.py', run_name='__main__')"])
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not line:
        raise SystemExit(f"arm {arm!r} failed:\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    d = json.loads(line[-1])
    return d["ms_per_step"], d["value"]


def main():
    argv = sys.argv[1:]
    rounds = 2
    if argv[:1] == ["--rounds"]:
        rounds, argv = int(argv[1]), argv[2:]
    i = argv.index("--") if "--" in argv else len(argv)
    arms, bench_args = argv[:i], argv[i + 1:]
    res = {a: [] for a in arms}
    for _ in range(rounds):
        for a in arms:
            ms, v = run(a, bench_args)
            res[a].append(ms)
            print(f"{a or 'default':45s} {ms:8.3f} ms/step {v:12,.0f} tok/s", flush=True)
    for a in arms:
        print(f"mean {a or 'default':40s} {sum(res[a]) / len(res[a]):8.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
