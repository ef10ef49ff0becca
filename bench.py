"""Benchmark: BLS12-377 G1 MSM throughput on MI355X (BASELINE.json configs[1]),
plus the sqrt-PST commit+open seconds at 2^20 (configs[2]) and 2^24
(configs[3]) variables, with the C++ CPU restatement timed beside them.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A step = one variable-base G1 MSM over 2^20 points (canonical Fr scalars,
Montgomery affine bases, both resident in HBM before the timed region) -- the
`msm_unchecked` of sqrt_pst.rs:198 / mipp.rs:393 at BASELINE's size.

N > 1: one process per GPU.  Run directly (`--gpus N` without WORLD_SIZE in
the environment) this script starts `torch.distributed.run` with N ranks as a
child process before it touches the GPU and relays its exit code; launched
by torch.distributed.run it reads RANK / LOCAL_RANK / WORLD_SIZE.  Every rank
runs its own MSMs (weak scaling, no data-path collective); the timed region
is bracketed by barrier + synchronize, the max over ranks is taken, and rank 0
prints ONE JSON line.  The 2^24 leg shards the commit's rows over the ranks:
each rank uploads only its column block of Z (one 2D copy), commits its rows
and the Miller loops of their IPP pairs, one RCCL all-gather moves [row
commitments | Miller partial], rank 0 runs the final exponentiation and the
(transcript-sequential) open.

roofline: the dominant kernel is bucket accumulation (k_bucket_acc_short_lds, one
launch per window group, msm.hip msm_groups); its duration per MSM (all group
launches, back to back on the library's own stream, with the earlier groups'
reductions running beside them on aux streams) is measured with HIP events on
that stream over the timed region (tpst_profile_*).  Algorithmic bytes per MSM =
128 B per scalar-point pair (32 B Fr + 96 B affine G1).  The
kernel is integer-VALU bound ("bound": "valu-int32"), so the HBM fraction is
small by construction; `traffic` is the rocprofv3 PMC HBM bytes per launch of
the same kernel (profiles/, FETCH_SIZE x2 + WRITE_SIZE per the gfx950
correction), `compute` the VALU issue rate from SQ_INSTS_VALU and the Fq-mul
rate against the measured microbenchmark peak.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "PST commit+open sec, 2^20-var poly BLS12-377; G1 MSM Mscalar/s at 1/2/4/8 GPU"
LOG_N = 20
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
BYTES_PER_PAIR = 128           # 32 B scalar + 96 B affine base
# the accumulation's Fq product (field29.h, 13 x 29-bit limbs): 13 x 13 a*b + 12 x 13 m*p limb
# products, one v_mad_u64_u32 each (p_0 = 1 makes the m_k * p_0 terms adds)
LIMB_PRODUCTS_PER_FQ_MUL = 325
MB_FQMUL_KIND = 12  # tpst_microbench kind of that product (kind 0: field.h's 12 x 32-bit product)
SEED = 0x7E57D0
def _latest(*rel):
    """The newest round's copy of a committed profile file (profiles/r06 first)."""
    for r in ("r06", "r05/final", "r03"):
        f = os.path.join(ROOT, "profiles", r, *rel)
        if os.path.exists(f):
            return f
    return os.path.join(ROOT, "profiles", "r06", *rel)


PMC_FILE = _latest("pmc_bucket_acc_short.json")
PMC_FILE_K1 = _latest("pmc_bucket_acc_chunk_2p24.json")
# VALU issue-slot passes (tools/pmc_valu.py): SQ_INSTS_VALU + SQ_INSTS_VALU_INT64
PMC_VALU_K2 = _latest("pmc_valu_k2.json")
PMC_VALU_K1 = _latest("pmc_valu_k1.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=LOG_N)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-pst", action="store_true", help="skip the sqrt-PST commit+open leg")
    ap.add_argument("--pst-log-n", type=int, default=20)
    ap.add_argument("--no-sharded", action="store_true", help="skip the 2^24 (row-sharded) commit+open leg")
    ap.add_argument("--sharded-log-n", type=int, default=24)
    ap.add_argument("--no-r1cs", action="store_true", help="skip the R1CSProof::prove leg")
    ap.add_argument("--r1cs-log-cons", type=int, default=20)
    ap.add_argument("--no-groth16", action="store_true", help="skip the Groth16 prove leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launcher / rendezvous / timing plumbing only (gloo)")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """--gpus N from a plain invocation: start N ranks under torch.distributed.run
    as a CHILD process (nothing here has touched the GPU) and return its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, _cpu_threads() // args.gpus)))
    return subprocess.run(cmd, env=env).returncode


def _cpu_threads():
    """Cores this job may use: the affinity mask, capped by OMP_NUM_THREADS when
    the environment sets it (the GPU box gives each GPU job a 16-core share)."""
    n = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def fq_mults_per_madd(pmc=None):
    """Fq-product equivalents of one XYZZ mixed add: counted (SQ_INSTS_VALU of
    the accumulation per madd over that of the Fq-multiply microbenchmark per
    product, tools/pmc_summary.py) when the round's PMC file holds it, else the
    formula's 8M + 2S plus ~2 products' worth of modular adds."""
    if pmc and pmc.get("fq_mul_equiv_per_madd"):
        return float(pmc["fq_mul_equiv_per_madd"])
    return 12.0


def valu_slots(path, kernel_ms, rates):
    """VALU issue-slot fraction of an accumulation kernel from its committed
    PMC pass (tools/pmc_valu.py: SQ_INSTS_VALU + SQ_INSTS_VALU_INT64 slots per
    launch group, v_mad_u64_u32 counting two) over this run's kernel time,
    against the live-measured v_add_u32 issue rate (one slot per instruction)."""
    if not os.path.exists(path):
        return {}
    try:
        d = json.load(open(path))
    except ValueError:
        return {}
    slots = d.get("issue_slots")
    if not slots or not kernel_ms:
        return {}
    rate = slots / (kernel_ms * 1e-3)
    return {"valu_slots_per_group": slots, "valu_int64_frac": round(d.get("int64_frac_of_valu") or 0.0, 4),
            "valu_slot_frac": round(rate / rates["v_add_u32"], 4),
            "valu_busy_frac_pmc": round(d["valu_busy_frac"], 4) if d.get("valu_busy_frac") else None,
            "valu_utilization_pmc": round(d["valu_utilization"], 4) if d.get("valu_utilization") else None,
            "valu_slots_source": os.path.relpath(path, ROOT),
            "valu_slot_note": ("slots = SQ_INSTS_VALU + SQ_INSTS_VALU_INT64 (v_mad_u64_u32 issues over two slots) "
                               "per launch group of the PMC pass / this run's kernel time, over the measured "
                               "v_add_u32 chip issue rate")}


def issue_rates(ctx):
    """Chip-wide wave-instruction issue rates (per s) of v_mad_u64_u32 and
    v_add_u32 (microbench kinds 6 and 9: 8 independent chains per lane, 8
    waves per SIMD), measured live (tools/mb_wave.py does the same sweep)."""
    out = {}
    thr, iters = 256 * 4 * 8 * 64, 2000
    for kind, name in ((6, "v_mad_u64_u32"), (9, "v_add_u32")):
        ctx.microbench(kind, 64, 4)
        ms = min(ctx.microbench(kind, thr, iters) for _ in range(3))
        out[name] = thr / 64 * iters * 32 / (ms * 1e-3)
    return out


def _stage_ms(ctx):
    """Average device span (ms) per recorded stage since the last reset."""
    return {k: round(v[0] / v[1], 4) for k, v in ctx.profile_read().items() if v[1]}


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def _max_over_ranks(dist, dev, x):
    import torch
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if dist.get_backend() == "gloo" else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def dry_run(args):
    """CPU rehearsal of the multi-rank plumbing (tests/test_distributed.py):
    gloo rendezvous, barrier-bracketed timing, max over ranks, one JSON line."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    else:
        dist = None
    for _ in range(args.warmup):
        time.sleep(0.001)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))  # ranks finish at different times: the max must win
    if dist:
        dist.barrier()
    el = _max_over_ranks(dist, "cpu", time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "Mscalar/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dry_run": True,
                          "config": {"workload": "dry run (no GPU)"}}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args)
    if args.dry_run:
        return dry_run(args)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("TPST_BENCH_SHARED_GPU") == "1":
            # rehearsal of the multi-rank path on a box with fewer GPUs than
            # ranks: ranks share cards and talk over gloo (RCCL refuses two
            # ranks on one GPU); timings are not scaling numbers
            local %= max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl")
    from testudo_amd import Context
    from testudo_amd.sqrt_pst import fr_stream

    ctx = Context(local)
    n = 1 << args.log_n
    dev = torch.device("cuda", local)
    # synthetic inputs: uniform Fr scalars, bases b_i * G (distinct points)
    sc, _ = fr_stream(SEED + 17 * rank, n)
    bk, _ = fr_stream(SEED + 1000 + 17 * rank, n)
    d_sc = torch.from_numpy(sc.view(np.int64)).to(dev)
    d_bk = torch.from_numpy(bk.view(np.int64)).to(dev)
    d_bases = torch.empty(n * 12, dtype=torch.int64, device=dev)
    d_out = torch.empty(12, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctx.g1_mul_generator_dev(d_bk.data_ptr(), n, d_bases.data_ptr())
    ctx.synchronize()

    def step():  # the pipelined entry point (tpst_g1_msm_dev_async): consecutive MSMs overlap
        ctx.g1_msm_dev_async(d_bases.data_ptr(), d_sc.data_ptr(), n, d_out.data_ptr())

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.profile_reset()
    ctx.profile(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.profile(False)
    stages = ctx.profile_read()
    elapsed = _max_over_ranks(dist, dev, t1 - t0)
    # one MSM alone (synchronised after each call): the latency; the timed
    # loop above overlaps call i's latency-bound tail with call i+1
    # (tpst_g1_msm_dev pipelining)
    lat = []
    for _ in range(5):
        ctx.synchronize()
        ta = time.perf_counter()
        step()
        ctx.synchronize()
        lat.append(time.perf_counter() - ta)
    latency_ms = sorted(lat)[len(lat) // 2] * 1e3

    # correctness spot check of this rank's result against the size-independent
    # property MSM(b_i G) = (sum s_i b_i) G, verified with the library's
    # generator multiplication (a different code path from the MSM)
    out = d_out.cpu().numpy().view(np.uint64)
    from testudo_amd.encoding import fr_array
    R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
    s_int = sc.astype(object)
    b_int = bk.astype(object)
    sv = s_int[:, 0] + (s_int[:, 1] << 64) + (s_int[:, 2] << 128) + (s_int[:, 3] << 192)
    bv = b_int[:, 0] + (b_int[:, 1] << 64) + (b_int[:, 2] << 128) + (b_int[:, 3] << 192)
    tot = int(np.dot(sv, bv) % R)
    parity_ok = bool(np.array_equal(out, ctx.g1_mul_generator(fr_array([tot]))[0]))

    sharded = sharded20 = split = None
    if dist is not None:  # every rank takes part in the multi-rank legs
        try:
            split = split_msm_leg(ctx, n, dist, dev, args.steps, args.warmup, out)
        except Exception as e:
            split = {"error": repr(e)}
        if not args.no_pst:
            try:
                sharded20 = sharded_leg(ctx, args.pst_log_n, dist, dev)
            except Exception as e:
                sharded20 = {"error": repr(e)}
        if not args.no_sharded:
            try:
                sharded = sharded_leg(ctx, args.sharded_log_n, dist, dev)
            except Exception as e:
                sharded = {"error": repr(e)}
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    ms_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed / 1e6  # Mscalar/s, whole job
    acc_ms, acc_cnt = stages["bucket_acc"]
    acc_avg_ms = acc_ms / max(acc_cnt, 1)
    alg_bytes = n * BYTES_PER_PAIR + 96
    achieved = alg_bytes / (acc_avg_ms * 1e-3) / 1e9
    pmc = None
    if os.path.exists(PMC_FILE):
        try:
            pmc = json.load(open(PMC_FILE))
        except ValueError:
            pmc = None
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    # compute roof, measured live on this GPU: the chip-wide issue rate of
    # v_mad_u64_u32 (one limb product) prices the accumulation's Fq product
    # at its 325 limb products -- the multiply-issue roof; the Fq-product
    # microbenchmark (same product) is the achieved-in-isolation rate;
    # v_add_u32's rate is the VALU issue peak
    rates = issue_rates(ctx)
    mad_roof_fqmul = rates["v_mad_u64_u32"] * 64 / LIMB_PRODUCTS_PER_FQ_MUL
    mb_threads = 256 * 16 * 64
    mb_iters = 200
    ctx.microbench(MB_FQMUL_KIND, mb_threads, 10)  # warm: first launch loads the code object
    mb_fqmul = mb_threads * mb_iters / (min(ctx.microbench(MB_FQMUL_KIND, mb_threads, mb_iters)
                                            for _ in range(3)) * 1e-3)
    c_bits = 16
    windows = 8  # GLV: two 127-bit halves, 8 signed 16-bit windows each
    madds = 2 * n * windows
    fq_per_madd = fq_mults_per_madd(pmc)
    achieved_fqmul = madds * fq_per_madd / (acc_avg_ms * 1e-3)
    compute = {"bound": "valu-int32", "kernel": "k_bucket_acc_short_lds<2, true>",
               "roof": "v_mad_u64_u32 issue (measured) / %d limb products per Fq product" % LIMB_PRODUCTS_PER_FQ_MUL,
               "mad_wave_insts_per_s": rates["v_mad_u64_u32"], "peak_fq_mul_per_s": mad_roof_fqmul,
               "achieved_fq_mul_per_s": achieved_fqmul, "frac": round(achieved_fqmul / mad_roof_fqmul, 4),
               "microbench_fq_mul_per_s": mb_fqmul, "microbench_frac": round(mb_fqmul / mad_roof_fqmul, 4),
               "achieved_vs_microbench": round(achieved_fqmul / mb_fqmul, 4),
               "fq_mul_per_madd": round(fq_per_madd, 3),
               "fq_mul_per_madd_source": ("SQ_INSTS_VALU ratio, " + os.path.relpath(PMC_FILE, ROOT))
               if pmc and pmc.get("fq_mul_equiv_per_madd") else "formula (8M + 2S + adds)"}
    if pmc and pmc.get("valu_insts_per_launch"):
        rate = pmc["valu_insts_per_launch"] / (acc_avg_ms * 1e-3)
        compute.update({"valu_wave_insts_per_msm": pmc["valu_insts_per_launch"],
                        "valu_issue_per_s": rate, "valu_issue_peak_per_s": rates["v_add_u32"],
                        "valu_issue_peak_source": "v_add_u32 chip issue rate, measured",
                        "valu_issue_frac": round(rate / rates["v_add_u32"], 4),
                        "valu_issue_frac_note": "instructions, not issue slots (v_mad_u64_u32 = 2 slots)"})
    compute.update(valu_slots(PMC_VALU_K2, acc_avg_ms, rates))

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mscalar/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (SplitMix64 uniform Fr scalars, bases b_i*G1 generated on device)",
        "config": {"workload": "single BLS12-377 G1 Pippenger MSM, 2^%d points per GPU (BASELINE configs[1])"
                               % args.log_n,
                   "n_points": n, "curve": "BLS12-377 G1", "window_bits": c_bits,
                   "parallelism": "independent MSM per rank" if world > 1 else "1 GPU"},
        "parity_ok": parity_ok,
        "latency_ms_single_call": round(latency_ms, 4),
        "pipelining": ("consecutive tpst_g1_msm_dev_async calls (the pipelined entry point; tpst_g1_msm_dev is "
                       "the stream-ordered one) overlap on three library streams with three arenas: "
                       "call i+1's scalar decomposition and sort run under call i's bucket accumulation, its "
                       "accumulation under call i's last-window-group tail (fixup, bucket reduction, window chain, "
                       "affine output); ms_per_step is the steady state, latency_ms_single_call one call "
                       "synchronised alone"),
        "stages_ms_per_step": {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items() if v[1]},
        "roofline": {"bound": "valu-int32", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                     "traffic_source": (os.path.relpath(PMC_FILE, ROOT) if pmc else None),
                     "kernel": "k_bucket_acc_short_lds (G1, 128-B records staged through LDS; 3 window-group launches per MSM)",
                     "alg_bytes_per_msm": alg_bytes, "kernel_ms_per_msm": round(acc_avg_ms, 4), "launches_per_msm": 3,
                     "note": ("per MSM = the sum over its 3 window-group launches (bytes and time alike, so achieved "
                              "is the per-launch ratio); HBM column secondary: the kernel is bound by 32-bit integer "
                              "VALU issue (compute.valu_slot_frac)")},
        "compute": compute,
    }
    if world > 1 and os.environ.get("TPST_BENCH_SHARED_GPU") == "1":
        result["rehearsal"] = ("%d ranks sharing %d GPU(s) over gloo (TPST_BENCH_SHARED_GPU=1): a correctness "
                               "rehearsal of the multi-rank legs; the timings are NOT scaling numbers"
                               % (world, max(1, torch.cuda.device_count())))
    if split is not None:
        result["msm_split"] = split
    if sharded20 is not None:
        result["pst"] = sharded20
    if sharded is not None:
        result["pst_2p24"] = sharded
    if not args.no_pst and world == 1:
        result["pst"] = pst_leg(ctx, args.pst_log_n)
    if dist is None and not args.no_sharded:
        try:
            result["pst_2p24"] = sharded_leg(ctx, args.sharded_log_n, None, dev)
        except Exception as e:  # never lose the bench line to the secondary leg
            result["pst_2p24"] = {"error": repr(e)}
    if not args.no_r1cs and world == 1:
        try:
            result["r1cs"] = r1cs_leg(ctx, args.r1cs_log_cons)
        except Exception as e:  # never lose the bench line to the secondary leg
            result["r1cs"] = {"error": repr(e)}
    if not args.no_groth16 and world == 1:
        try:
            result["groth16"] = groth16_leg(ctx, args.r1cs_log_cons)
        except Exception as e:  # never lose the bench line to the secondary leg
            result["groth16"] = {"error": repr(e)}
    if not args.no_cpu:  # rank 0 (at N > 1 the other ranks wait at the closing barrier)
        result["cpu_baseline"] = cpu_leg(ctx, bk, sc, out, result)
    print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def pst_leg(ctx, log_n, reps=5):
    """sqrt-PST commit + open at 2^log_n variables (BASELINE configs[2]),
    timed like benches/pst.rs:52-62 (eval / get_q before the open timer):
    the median of `reps` warm runs.  Also reported: the H2D upload of Z
    (from_evaluations; BASELINE.md's GPU-time definition includes it),
    commit+open including it, and the device spans of one further, profiled
    run under the reference's Timer labels (hipEvents on the library's streams:
    first command to last, host launch overhead excluded)."""
    from testudo_amd import sqrt_pst as S
    nv = (log_n + 1) // 2
    t = time.perf_counter()
    S.srs_setup(ctx, nv, SEED + 1)
    setup_s = time.perf_counter() - t
    Z, k = S.fr_stream(SEED, 1 << log_n)
    pt, _ = S.fr_stream(SEED, log_n, k)
    # the first commit+open of the process (cold: code objects load, scratch
    # arenas grow) is reported separately; then the median of `reps` warm runs
    runs = []
    for rep in range(reps + 2):
        prof = rep == reps + 1  # the last run: device spans only, not timed
        ctx.synchronize()
        t = time.perf_counter()
        pl = S.Polynomial.from_evaluations(ctx, Z)
        h2d_s = time.perf_counter() - t
        if prof:
            ctx.profile_reset()
            ctx.profile(True)
        t = time.perf_counter()
        comms, T = pl.commit()
        commit_s = time.perf_counter() - t
        v = pl.eval(pt)
        tr = S.PoseidonTranscript()
        t = time.perf_counter()
        U, pst_proof, mipp = pl.open(tr, comms, pt, T)
        open_s = time.perf_counter() - t
        if prof:
            ctx.profile(False)
            spans = _stage_ms(ctx)
        else:
            runs.append((commit_s, open_s, h2d_s))
    _PST_LAST[log_n] = {"comms": comms, "T": T, "U": U, "comms_t": mipp.comms_t}
    cold = runs[0]
    warm = runs[1:]
    c, o, h = (_median([r[i] for r in warm]) for i in range(3))
    co = _median([r[0] + r[1] for r in warm])
    t = time.perf_counter()
    ok = S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
    verify_s = time.perf_counter() - t
    sizes = _wire_sizes(ctx, nv, pst_proof, mipp)
    env_tab = os.environ.get("TPST_COMMIT_TABLE")
    in_commit = env_tab != "0"
    return {"log_n": log_n, "commit_s": round(c, 4), "open_s": round(o, 4), **sizes,
            "fold_table_in_commit": in_commit,
            "fold_table_note": ("the opening's GLV fold table over comm_list is built by the commit (beside its "
                                "IPP): open_s excludes it, commit_plus_open_s is the comparable total"
                                if in_commit else "the opening builds its fold table (inside open_s)"),
            "commit_plus_open_s": round(co, 4), "reps": reps, "timing": "median of the warm reps",
            "h2d_s": round(h, 4), "commit_open_incl_h2d_s": round(co + h, 4),
            "device_commit_s": round(spans.get("sqrt_commit", 0.0) * 1e-3, 5),
            "device_open_s": round(spans.get("sqrt_open", 0.0) * 1e-3, 5),
            "stages_ms": {k: spans[k] for k in ("comm_list", "ipp", "sqrt_commit", "msm", "mipp_prove", "pst_open",
                                                "sqrt_open", "batch_sort", "bucket_acc") if k in spans},
            "first_call": {"commit_s": round(cold[0], 4), "open_s": round(cold[1], 4)},
            "verify_s": round(verify_s, 4), "srs_setup_s": round(setup_s, 3), "verified": ok,
            "note": "Z resident in HBM for commit_s/open_s (benches/pst.rs:48-62: the polynomial is built before "
                    "the timers); h2d_s = from_evaluations from pageable host memory; eval before the open timer; "
                    "SRS tables built in srs_setup; device_*_s / stages_ms = hipEvent spans of one extra profiled "
                    "run (reference Timer labels, sqrt_pst.rs:118-228)"}


_R1CS_LAST = None
_PST_LAST = {}  # log_n -> the GPU legs' commitments and proof parts, for the CPU leg's parity check


def r1cs_leg(ctx, log_cons, reps=3):
    """R1CSProof::prove (r1csproof.rs:237-370, Groth16 step excluded) on a
    synthetic 2^log_cons-constraint instance with as many variables: the live
    equivalent of BASELINE configs[4] (testudo_snark::prove is absent from the
    reference snapshot).  Witness commit + both sum-checks +
    the PST opening, instance and SRS built before the timer."""
    from testudo_amd import r1cs as D
    from testudo_amd import sqrt_pst as S
    n_cons = n_vars = 1 << log_cons
    S.srs_setup(ctx, (log_cons + 1) // 2, SEED + 1)
    inst, vars_, inputs = D.R1CSInstance.produce_synthetic_r1cs(ctx, n_cons, n_vars, 10, SEED + 7)
    times = []
    for _ in range(reps + 1):
        ctx.synchronize()
        t = time.perf_counter()
        proof, rx, ry = D.R1CSProof.prove(inst, vars_, inputs, S.PoseidonTranscript())
        times.append(time.perf_counter() - t)
    # R1CSInstance::commit (SPARK dense representation + Hyrax commitments), the
    # SNARK's preprocessing -- not part of prove; timed once warm
    inst.commit(b"gens_r1cs_eval")
    t = time.perf_counter()
    ops, mem = inst.commit(b"gens_r1cs_eval")
    commit_s = time.perf_counter() - t
    from testudo_amd.encoding import limbs_to_int
    global _R1CS_LAST
    _R1CS_LAST = {"log_cons": log_cons, "seed": SEED + 7, "proof": proof}
    R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
    az, bz, cz, azbz = [limbs_to_int(x) for x in proof.claims_phase2]
    return {"num_cons": n_cons, "num_vars": n_vars, "num_inputs": 10, "prove_s": round(sorted(times[1:])[reps // 2], 4),
            "first_call_s": round(times[0], 4), "reps": reps, "claims_consistent": azbz == az * bz % R,
            "instance_commit_s": round(commit_s, 4), "instance_commit_rows": [len(ops), len(mem)],
            "note": "R1CSProof::prove minus prove_verifier (Groth16): witness sqrt-PST commit, phase-one cubic and "
                    "phase-two quad sum-checks on the device, PST opening at ry[1..]; instance + SRS set up "
                    "before the timer"}


def groth16_leg(ctx, log_cons, reps=3):
    """Groth16::prove (r1csproof.rs:421, ark-groth16 LibsnarkReduction) over the
    synthetic 2^log_cons-constraint R1CS instance with as many variables:
    witness map (7 NTTs over the 2^(log_cons+1) domain) + four device MSMs
    (A: G1, B: G2 and G1, C: G1 over L, H and the constants).  Key generation
    before the timer; the proof checked by the pairing equation."""
    from testudo_amd import groth16 as D
    from testudo_amd import r1cs as S
    from testudo_amd.encoding import fr_array
    n_cons = n_vars = 1 << log_cons
    inst, vars_, inputs = S.R1CSInstance.produce_synthetic_r1cs(ctx, n_cons, n_vars, 10, SEED + 7)
    t = time.perf_counter()
    pk = D.ProvingKey.setup(inst, fr_array([SEED + 11, SEED + 12, SEED + 13, SEED + 14, SEED + 15]))
    ctx.synchronize()
    setup_s = time.perf_counter() - t
    r, s = fr_array([SEED + 21]), fr_array([SEED + 22])
    times = []
    for _ in range(reps + 1):
        ctx.synchronize()
        t = time.perf_counter()
        proof = D.prove(pk, inst, vars_, inputs, r, s)
        times.append(time.perf_counter() - t)
    t = time.perf_counter()
    ok = D.verify(ctx, pk.vk(), inputs, proof)
    verify_s = time.perf_counter() - t
    return {"num_cons": n_cons, "num_vars": n_vars, "num_inputs": 10, "domain": pk.domain_size,
            "prove_s": round(sorted(times[1:])[reps // 2], 4), "first_call_s": round(times[0], 4), "reps": reps,
            "setup_s": round(setup_s, 3), "verify_s": round(verify_s, 4), "verified": ok,
            "note": "Groth16 prover of the R1CS instance itself (the reference proves its verifier circuit, "
                    "constraints.rs, out of scope); toxic waste and (r, s) fixed; key generation before the timer"}


def _wire_sizes(ctx, nv, pst_proof, mipp):
    """benches/pst.rs:43-46,64-74: compressed CanonicalSerialize lengths."""
    from testudo_amd import serialize as W
    from testudo_amd import sqrt_pst as S
    return {"proof_size": W.proof_size(pst_proof, mipp),
            "commiter_key_size": len(W.ser_committer_key(nv, S.srs_export(ctx, nv)))}


def sharded_leg(ctx, log_n, dist, dev, reps=5):
    """sqrt-PST commit + open at 2^log_n variables (BASELINE configs[3] at
    2^24; configs[2] at 2^20 when N > 1).
    N > 1: every rank uploads only its column block of Z and commits its rows
    AND their share of the IPP's Miller loops (one all-gather of [row
    commitments | Miller partial] device buffers, one final exponentiation on
    rank 0, read from the gathered buffer); then each rank computes its rows'
    share of get_q's z_q and of c_u (one all-gather, summed on rank 0 -- the
    q / eval step that benches/pst.rs runs before the open timer), and rank 0
    opens from q with the MIPP rounds split over the ranks while a round has
    >= 4 rows per rank (tpst_poly_open_sharded: every rank folds, pairs and
    cross-multiplies its own rows, one all-gather per product; rank 0 alone
    for the last rounds, the PST proof of q and the final folds; SURVEY.md
    §8(e)).  No rank holds the whole Z.  N = 1: the plain commit + open.
    Timing as BASELINE.md:43-45: the median of `reps` warm runs (commit and
    open: max over ranks), plus the H2D upload of Z; then one profiled run for
    the device spans and K1's roofline (the dominant kernel of the commit)."""
    from testudo_amd import sqrt_pst as S
    from testudo_amd.distributed import (TorchExchange, shard_rows, sharded_commit, sharded_open, sharded_open_inputs,
                                         sharded_rounds)
    nv = (log_n + 1) // 2
    t = time.perf_counter()
    S.srs_setup(ctx, nv, SEED + 1)
    setup_s = time.perf_counter() - t
    Z, k = S.fr_stream(SEED, 1 << log_n)
    pt, _ = S.fr_stream(SEED, log_n, k)
    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    r0, r1 = shard_rows(1 << (log_n // 2), world, rank)
    if dist:
        dist.barrier()
    t = time.perf_counter()
    if dist:  # the rank-local column block only
        shard = S.Polynomial.from_evaluations_cols(ctx, Z, r0, r1)
    else:
        shard = S.Polynomial.from_evaluations(ctx, Z)
    ctx.synchronize()
    h2d_s = _max_over_ranks(dist, dev, time.perf_counter() - t)
    del Z
    xch = TorchExchange(ctx, dist, dev, log_n) if dist else None
    commits, qs, opens = [], [], []
    k1 = {}
    spans = {}
    for rep in range(reps + 2):
        prof = rep == reps + 1  # the last run: device spans only, not timed
        if dist:
            dist.barrier()
        ctx.synchronize()
        if prof:
            ctx.profile_reset()
            ctx.profile(True)
        t = time.perf_counter()
        if dist:
            comms, T, own = sharded_commit(log_n, shard.commit_rows_partial_into,
                                           lambda got: S.gt_final_exp_product_gathered(ctx, got, r1 - r0), dist, dev)
        else:
            comms, T = shard.commit()
        ctx.synchronize()
        if dist:
            dist.barrier()
        c_el = _max_over_ranks(dist, dev, time.perf_counter() - t)
        if prof:
            ctx.profile(False)
            k1 = _stage_ms(ctx)
        else:
            commits.append(c_el)
        # q (and c_u) before the open timer, as eval does in benches/pst.rs:48-62
        t = time.perf_counter()
        if dist:
            zq, U = sharded_open_inputs(log_n, lambda a, b, out: shard.get_q_partial_into(pt, a, b, out),
                                        lambda a, b: S.cu_partial(ctx, log_n, pt, a, b, own),
                                        lambda got: S.fr_sum(ctx, got), lambda sh: S.g1_sum(ctx, sh), dist, dev)
            pl = S.Polynomial.from_q(ctx, log_n, pt, zq, U) if rank == 0 else None
        else:
            pl = shard
        v = pl.eval(pt) if rank == 0 else None
        ctx.synchronize()
        if dist:
            dist.barrier()
        q_el = _max_over_ranks(dist, dev, time.perf_counter() - t)
        if not prof:
            qs.append(q_el)
        if dist:  # the MIPP rounds on every rank's rows (C4), then rank 0 alone
            dist.barrier()
        if prof and rank == 0:
            ctx.profile_reset()
            ctx.profile(True)
        t = time.perf_counter()
        if dist:
            out = sharded_open(ctx, log_n, pl, comms, pt, U, S.PoseidonTranscript(), dist, dev, exchange=xch)
            if rank == 0:
                U, pst_proof, mipp = out
        else:
            U, pst_proof, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
        o_el = _max_over_ranks(dist, dev, time.perf_counter() - t)
        if prof:
            if rank == 0:
                ctx.profile(False)
                spans = _stage_ms(ctx)
        else:
            opens.append(o_el)
    if dist:
        dist.barrier()
    if rank != 0:
        return None
    ok = S.verify(ctx, S.PoseidonTranscript(), U, pt, v, pst_proof, mipp, T)
    _PST_LAST[log_n] = {"comms": comms, "T": T, "U": U, "comms_t": mipp.comms_t}
    warm = list(zip(commits[1:], opens[1:]))
    c, o = _median([w[0] for w in warm]), _median([w[1] for w in warm])
    co = _median([w[0] + w[1] for w in warm])
    res = {"log_n": log_n, "commit_s": round(c, 4), "open_s": round(o, 4), "commit_plus_open_s": round(co, 4),
           "reps": reps, "timing": "median of the warm reps (commit: max over ranks)",
           "h2d_s": round(h2d_s, 4), "commit_open_incl_h2d_s": round(co + h2d_s, 4),
           "device_commit_rank0_s": round(k1.get("sqrt_commit", 0.0) * 1e-3, 5) if world == 1 else None,
           "device_open_s": round(spans.get("sqrt_open", 0.0) * 1e-3, 5),
           "stages_ms": {**{k: k1[k] for k in ("comm_list", "ipp", "sqrt_commit", "batch_sort", "bucket_acc")
                            if k in k1},
                         **{k: spans[k] for k in ("msm", "mipp_prove", "pst_open", "sqrt_open") if k in spans}},
           **_wire_sizes(ctx, nv, pst_proof, mipp),
           "first_call": {"commit_s": round(commits[0], 4), "open_s": round(opens[0], 4)},
           "q_eval_s": round(_median(qs[1:]), 4),
           "ranks": world, "rows_per_rank": r1 - r0, "verified": ok, "srs_setup_s": round(setup_s, 3),
           "exchange": ("per-rank column-block upload; %s all_gather of [96-B row commitments | 576-B Miller "
                        "partial] device buffers, FE on rank 0; %s all_gather of [z_q share | c_u share], mod-r / "
                        "G1 sum; sharded MIPP open: %d all_gathers (cross XYZZ partials, Miller partials) on the "
                        "library's comm stream, the last %d rounds on rank 0"
                        % ((("RCCL" if dist.get_backend() == "nccl" else "gloo"),) * 2
                           + (xch.calls // (reps + 2), log_n // 2 - sharded_rounds(log_n, world))))
                        if dist else "none"}
    if "bucket_acc" in k1:  # K1 (k_bucket_acc_chunk + fixup) over this rank's rows
        rows = r1 - r0
        npts = 1 << (log_n - log_n // 2)
        alg = rows * npts * 32 + npts * 96 + rows * 96  # scalars + bases once + row outputs
        acc_s = k1["bucket_acc"] * 1e-3
        pmc = None
        if os.path.exists(PMC_FILE_K1):
            try:
                pmc = json.load(open(PMC_FILE_K1))
            except ValueError:
                pmc = None
        # the PMC files hold the one-GPU 2^24 commit (4096 rows): quoted only
        # when this rank accumulates the same rows
        same = pmc is not None and world == 1 and log_n == 24
        res["roofline_k1"] = {"bound": "valu-int32 / random gathers", "kernel": "k_bucket_acc_chunk_lds + fixup",
                              "achieved": round(alg / acc_s / 1e9, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(alg / acc_s / 1e9 / HBM_PEAK_GBS, 6), "alg_bytes_per_launch": alg,
                              "kernel_ms": round(k1["bucket_acc"], 4),
                              "traffic": pmc.get("hbm_bytes_per_launch") if same else None,
                              "traffic_source": os.path.relpath(PMC_FILE_K1, ROOT) if same else None,
                              "gather_bytes_per_launch": pmc.get("gather_bytes_per_launch") if same else None}
        if world == 1 and log_n == 24:
            res["roofline_k1"].update(valu_slots(PMC_VALU_K1, k1["bucket_acc"], issue_rates(ctx)))
    return res


def split_msm_leg(ctx, n, dist, dev, steps, warmup, ref_out):
    """Strong scaling of ONE 2^log_n G1 MSM (sqrt_pst.rs:198 / mipp.rs:393):
    rank g takes points [g n/N, (g+1) n/N) of rank 0's inputs, computes its
    share as a raw XYZZ sum, one all-gather moves the 192-B shares and rank 0
    sums them on the device (testudo_amd/distributed.py sharded_msm).  Timed
    like the headline: barrier + synchronize around `steps` MSMs, max over
    ranks; checked against rank 0's single-GPU MSM of the same inputs."""
    import torch
    from testudo_amd import sqrt_pst as S
    from testudo_amd.distributed import shard_rows, sharded_msm
    from testudo_amd.sqrt_pst import fr_stream
    world, rank = dist.get_world_size(), dist.get_rank()
    i0, i1 = shard_rows(n, world, rank)
    sc, _ = fr_stream(SEED, n)  # rank 0's inputs (bench.py main: SEED + 17 * 0)
    bk, _ = fr_stream(SEED + 1000, n)
    d_s = torch.from_numpy(sc[i0:i1].view(np.int64).copy()).to(dev)
    d_k = torch.from_numpy(bk[i0:i1].view(np.int64).copy()).to(dev)
    d_b = torch.empty((i1 - i0) * 12, dtype=torch.int64, device=dev)
    ctx.torch_to_lib()
    ctx.g1_mul_generator_dev(d_k.data_ptr(), i1 - i0, d_b.data_ptr())
    ctx.synchronize()

    def step():
        return sharded_msm(n, lambda a, b, o: S.g1_msm_partial_into(ctx, d_b.data_ptr(), d_s.data_ptr(), 0, b - a, o),
                           lambda got: S.g1_xyzz_combine(ctx, got), dist, dev)

    for _ in range(warmup):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = step()
    ctx.synchronize()
    torch.cuda.synchronize()
    dist.barrier()
    el = _max_over_ranks(dist, dev, time.perf_counter() - t0)
    if rank != 0:
        return None
    return {"value": round(n * steps / el / 1e6, 3), "unit": "Mscalar/s", "scaling": "strong",
            "ms_per_msm": round(el / steps * 1e3, 4), "n_points": n, "ranks": world, "points_per_rank": i1 - i0,
            "parity_ok": bool(np.array_equal(res.cpu().numpy().view(np.uint64), ref_out)),
            "exchange": "%s all_gather of the 192-B XYZZ shares, device sum on rank 0" % (
                "RCCL" if dist.get_backend() == "nccl" else "gloo")}


def cpu_leg(ctx, bk, sc, gpu_out, result):
    """C++ CPU restatement (oracle/cpu: arkworks-shaped msm_bigint_wnaf,
    OpenMP) on this host's cores: the 2^20 MSM, the 2^20 and the 2^24 sqrt-PST
    commit + open, each in full and checked against the GPU legs' outputs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "cpu"))
    import orc
    from testudo_amd import sqrt_pst as S
    threads = _cpu_threads()
    lib = orc.load()
    lib.orc_set_threads(threads)
    n = len(sc)
    bases = ctx.g1_mul_generator(bk)  # canonical affine, same points as the GPU run
    t = time.perf_counter()
    out = orc.g1_msm(bases, sc, parallel=True)
    dt = time.perf_counter() - t
    res = {"value": round(n / dt / 1e6, 4), "unit": "Mscalar/s", "cores": threads, "kind": "port",
           "sample": "full 2^%d-point G1 MSM (C++ restatement of ark-ec msm_bigint_wnaf, OpenMP over windows), "
                     "%.2f s" % (int(np.log2(n)), dt),
           "matches_gpu": bool(np.array_equal(out, gpu_out))}
    # sqrt-PST 2^20 commit + open, same inputs as the GPU leg
    try:
        lg = 20
        srs = orc.SRS((lg + 1) // 2, SEED + 1)
        Z, k = orc.fr_stream(SEED, 1 << lg)
        pt, _ = orc.fr_stream(SEED, lg, k)
        t = time.perf_counter()
        comms, T = orc.pst_commit(srs, Z, lg)
        c_s = time.perf_counter() - t
        t = time.perf_counter()
        orc.pst_open(srs, Z, lg, pt, comms)
        o_s = time.perf_counter() - t
        gpu = result.get("pst", {})
        res["pst"] = {"log_n": lg, "commit_s": round(c_s, 3), "open_s": round(o_s, 3),
                      "commit_plus_open_s": round(c_s + o_s, 3), "cores": threads,
                      "gpu_speedup": (round((c_s + o_s) / gpu["commit_plus_open_s"], 1)
                                      if gpu.get("commit_plus_open_s") else None),
                      "sample": "full 2^20 commit + open (open includes get_q, as orc.pst_open computes it)"}
        g20 = _PST_LAST.get(20)
        if g20 is not None:
            res["pst"]["matches_gpu"] = bool(np.array_equal(comms, g20["comms"]) and np.array_equal(T, g20["T"]))
        del Z
        # 2^24: the full commit + open (same inputs as the GPU 2^24 leg)
        lg = 24
        srs = orc.SRS((lg + 1) // 2, SEED + 1)
        Z, k = orc.fr_stream(SEED, 1 << lg)
        pt, _ = orc.fr_stream(SEED, lg, k)
        t = time.perf_counter()
        comms, T = orc.pst_commit(srs, Z, lg)
        c_s = time.perf_counter() - t
        t = time.perf_counter()
        pr = orc.pst_open(srs, Z, lg, pt, comms)
        o_s = time.perf_counter() - t
        gpu = result.get("pst_2p24", {})
        ent = {"log_n": lg, "commit_s": round(c_s, 3), "open_s": round(o_s, 3),
               "commit_plus_open_s": round(c_s + o_s, 3), "cores": threads,
               "gpu_speedup": (round((c_s + o_s) / gpu["commit_plus_open_s"], 1)
                               if gpu.get("commit_plus_open_s") else None),
               "sample": "full 2^24 commit (4096 row MSMs of 4096 points + 4096-pair IPP) + open (get_q, U, "
                         "12-round MIPP, PST open), measured"}
        g24 = _PST_LAST.get(24)
        if g24 is not None:
            ent["matches_gpu"] = bool(np.array_equal(comms, g24["comms"]) and np.array_equal(T, g24["T"])
                                      and np.array_equal(pr["U"], g24["U"])
                                      and np.array_equal(pr["comms_t"], g24["comms_t"]))
        res["pst_2p24"] = ent
        del Z
    except Exception as e:  # the headline CPU line must survive
        res["pst_error"] = repr(e)
    # R1CSProof::prove's sum-check section on the CPU (oracle/cpu, OpenMP) from
    # the GPU proof's T on: same transcript, so rx / ry must match exactly
    try:
        if _R1CS_LAST is not None:
            lc, pr = _R1CS_LAST["log_cons"], _R1CS_LAST["proof"]
            t = time.perf_counter()
            cpu = orc.r1cs_sumchecks(1 << lc, 1 << lc, 10, _R1CS_LAST["seed"], pr.T)
            sc_s = time.perf_counter() - t
            pst = res.get("pst", {})
            rr = {"num_cons": 1 << lc, "sumchecks_s": round(sc_s, 3), "cores": threads,
                  "matches_gpu": bool(np.array_equal(cpu["rx"], pr.rx) and np.array_equal(cpu["ry"], pr.ry)
                                      and np.array_equal(cpu["sc1"], pr.sc_proof_phase1)
                                      and np.array_equal(cpu["sc2"], pr.sc_proof_phase2)),
                  "sample": "full 2^%d-constraint sum-checks (eq tables, mat-vecs, phase one + two); prove_s = "
                            "this + the CPU 2^20 commit + open of the pst leg (same witness size)" % lc}
            if pst.get("commit_s") is not None and lc == 20:
                rr["prove_s"] = round(sc_s + pst["commit_s"] + pst["open_s"], 3)
                g = result.get("r1cs", {}).get("prove_s")
                rr["gpu_speedup"] = round(rr["prove_s"] / g, 1) if g else None
            res["r1cs"] = rr
    except Exception as e:
        res["r1cs_error"] = repr(e)
    return res


if __name__ == "__main__":
    sys.exit(main())
