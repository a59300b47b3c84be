#!/usr/bin/env python3
"""Headline benchmark: forward+logdetJ samples/s of the fused MI355X FlowChain
pass (BASELINE.json metric, configs[1]: d=5, 8 RealNVP layers, hidden 64,
batch 2^20 fp32 per GPU).

One "step" = one fused chain pass (df_chain_forward: x and ldj written) over
the rank's batch, inputs already resident in HBM.  Multi-GPU (torchrun, one
rank per GPU): every rank processes its own 2^20-sample shard (config 3:
8·2^20 over 8 GPUs) with no data-path collective — weak scaling; timing is the
max over ranks between barriers.  ``--mode nll`` benches the config-3 NLL step
instead (fused inverse + logpdf + fp64 Σ, then an RCCL all-reduce of
{Σ logpdf, count}).

Rank 0 prints ONE JSON line (bench contract).  Extra objects:
  roofline     — the fused kernel against the f32 MFMA peak (it is compute-
                 bound: 3,212 FLOP/B algorithmic intensity); achieved = 2·ΣMAC
                 per sample × samples per launch ÷ mean launch time from HIP
                 events on the launch stream.
  cpu_baseline — the C++/OpenMP fp32 restatement of the reference's CPU
                 forward (oracle/cpu_flow.cpp: Flux's unfused Dense order,
                 register-blocked GEMMs, one sample block per thread), pinned
                 to the numpy oracle by tests/test_oracle.py, timed on the
                 host cores on a bounded sample (rank 0, N=1 only); config 1
                 on its stated B = 4096 batches.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "forward+logdetJ Msamples/s, d=5 8-layer RealNVP, 1/2/4/8 MI355X"
PEAK_F32_TFLOPS = 157.3   # MI355X f32 MFMA dense peak (MI355X_MICROARCH.md)
# SPLIT kernel (df_uniform_impl.h): an f32 product as six bf16 MFMA products; bf16
# MFMA runs 16x the f32 MFMA rate (MI355X_MICROARCH.md § Matrix cores)
PEAK_SPLIT_TFLOPS = 16.0 * PEAK_F32_TFLOPS / 6.0
KERNELS = {0: "generic", 1: "specialised", 2: "specialised relu-only", 3: "FAST (exact f32 MFMA)",
           4: "FAST SPLIT (bf16x3 planes, 6 products on bf16 MFMA, f32 accumulate)", 5: "wide (exact f32 MFMA)",
           6: "wide SPLIT (bf16x3 planes, 6 products on bf16 MFMA, f32 accumulate)"}
PEAK_HBM_GBS = 8000.0
# HBM bytes per launch of the headline kernel from rocprofv3 PMC counters
# (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, WRITE_SIZE as is; KiB),
# measured on the headline workload and committed under profiles/.
TRAFFIC_PROFILES = {"cfg2": os.path.join("profiles", "r06final_pmc_cfg2.txt"),
                    "cfg4": os.path.join("profiles", "r06final_pmc_cfg4.txt")}


def source_sha16():
    """sha256 over the HIP/C++ sources of the product library, its header and its
    Makefile (per-unit compiler flags shape the kernels too): the PMC summaries record
    the one they profiled (tools/gpu_round4.sh)."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "densityflows.jl_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")))
    for f in files + ["../../include/densityflows_hip.h", "Makefile"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def pmc_summary(path):
    """traffic (HBM bytes per dispatch, gfx950 FETCH correction), MFMA busy and
    the profiled source hash from a committed PMC summary."""
    out = {"traffic": None, "mfma_busy": None, "source": None}
    try:
        vals = {}
        for line in open(os.path.join(ROOT, path)):
            if line.startswith("# source sha16"):
                out["source"] = line.split()[-1]
            parts = line.split()
            if len(parts) == 2 and parts[0] in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[parts[0]] = float(parts[1].replace(",", ""))
            if line.startswith("MFMA busy fraction"):
                out["mfma_busy"] = float(parts[-1])
        out["traffic"] = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    except Exception:
        pass
    return out


CONFIGS = {
    # name: (d, n, description)
    "cfg2": (5, 0, "config2: d=5, n=0, FlowChain(CouplingBlock, 4, 5; hidden 64) = 8 RealNVP layers, fp32"),
    "cfg1": (5, 1, "config1: d=5, n=1, README chain: 3 RNVP layers (masks [1,2,3],[3,4,5],[5,1,2], hidden 16) "
                   "+ NormalizationLayer(x, -1, 1), fp32"),
    "cfg4": (32, 8, "config4: d=32, n=8, FlowChain(CouplingBlock, 8, 32; n=8, hidden 256) = 16 RealNVP layers, fp32"),
}


def _init_nets(chain, rng):
    """Biases U(-0.1, 0.1); final Dense of each conditioner scaled by 0.1 so the
    deep random-init flows stay finite."""
    from densityflows_amd.layers import RNVPCouplingLayer, NICECouplingLayer, CouplingBlock

    def layers(e):
        if isinstance(e, CouplingBlock):
            return [e.layer_1, e.layer_2]
        if isinstance(e, (RNVPCouplingLayer, NICECouplingLayer)):
            return [e]
        return []

    for e in chain:
        for layer in layers(e):
            nets = [layer.t_net] + ([layer.s_net] if isinstance(layer, RNVPCouplingLayer) else [])
            for net in nets:
                for D in net:
                    D.b = ((rng.random(D.out_dim) * 2 - 1) * 0.1).astype(np.float32)
                net[-1].W = (net[-1].W * np.float32(0.1)).astype(np.float32)
    return chain


def build_chain(config="cfg2", seed=2):
    """Random-init model of a BASELINE config (Flux glorot_uniform weights)."""
    import densityflows_amd as dfa

    rng = np.random.default_rng(seed)
    if config == "cfg2":
        chain = dfa.FlowChain.repeat(dfa.CouplingBlock, 4, 5, hidden_dim_s=64, hidden_dim_t=64, rng=rng)
    elif config == "cfg4":
        chain = dfa.FlowChain.repeat(dfa.CouplingBlock, 8, 32, n=8, hidden_dim_s=256, hidden_dim_t=256, rng=rng)
    elif config == "cfg1":
        x = np.load(os.path.join(ROOT, "tests", "golden", "datatest_x.npy"))
        layers = [dfa.CouplingLayer(5, m, n=1, hidden_dim_s=16, hidden_dim_t=16, rng=rng)
                  for m in ([1, 2, 3], [3, 4, 5], [5, 1, 2])]
        chain = dfa.FlowChain(*layers, dfa.NormalizationLayer.from_data(x, -1.0, 1.0))
    else:
        raise SystemExit(f"unknown config {config}")
    return _init_nets(chain, rng)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(chain, d, n, seconds=12.0, sample=65536):
    """C++/OpenMP fp32 forward+logdetJ (oracle/cpu_flow.cpp) on the host cores,
    repeated passes over one `sample`-sample batch for ~`seconds`."""
    from oracle.cpu_flow import CPUFlow, max_threads

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or max_threads()
    f = CPUFlow(chain.to_spec(), d, n, np.float32)
    rng = np.random.default_rng(0)
    z = rng.standard_normal((d, sample)).astype(np.float32)
    th = rng.random((n, sample)).astype(np.float32)
    f.forward(z[:, :256], th[:, :256], threads)  # warm-up
    done, t0 = 0, time.perf_counter()
    win, w0, wdone = [], t0, 0       # per-window rates (~1 s each): the spread within this run
    while True:
        f.forward(z, th, threads)
        done += sample
        wdone += sample
        now = time.perf_counter()
        if now - w0 >= 1.0:
            win.append(wdone / (now - w0) / 1e6)
            w0, wdone = now, 0
        el = now - t0
        if el >= seconds:
            break
    win = sorted(win) or [done / el / 1e6]
    return {"value": done / el / 1e6, "unit": "Msamples/s", "cores": int(threads), "kind": "port",
            "cpu_model": cpu_model(),
            "spread_1s_windows": {"min": round(win[0], 4), "median": round(win[len(win) // 2], 4),
                                  "max": round(win[-1], 4), "windows": len(win),
                                  "note": "the host is shared: earlier rounds measured 4.5-7.2 Msamples/s on "
                                          "identical code across boxes (16 visible cores of a 64-core EPYC)"},
            "sample": f"{done} samples ({done // sample} passes of a {sample}-sample batch, C++/OpenMP fp32 "
                      f"restatement oracle/cpu_flow.cpp, {threads} threads) in {el:.1f} s"}


class _stdout_to_stderr:
    """fd 1 → fd 2 for a block (C-level prints such as RCCL's version banner)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def train_split_flops(chain, kernel_id):
    """FLOP per sample of one train! step (3F: forward, dX, dW) that the step's
    kernels run as bf16x3 split products, from the model's Dense shapes.

    Kernel 4 (FAST SPLIT, hidden <= 64 nets, fused per-net reverse kernel
    df_train_impl.h): forward first + hidden Dense, and the hidden Dense's W1ᵀδ and
    dW1 are split; W0ᵀδ, dW0, the output Dense GEMV, W_outᵀȳ and dW_out are f32.
    Kernel 6 (wide SPLIT, hidden 256, layer-wise reverse path df_ltrain.hip):
    the forward's three Denses and the hidden Dense's W1ᵀδ1 and dW1 are split,
    the rest f32.  Every other kernel: none."""
    from densityflows_amd.layers import RNVPCouplingLayer, NICECouplingLayer, CouplingBlock

    if kernel_id not in (4, 6):
        return 0.0
    nets = []
    for e in chain:
        for layer in ([e.layer_1, e.layer_2] if isinstance(e, CouplingBlock) else [e]):
            if isinstance(layer, RNVPCouplingLayer):
                nets += [layer.s_net, layer.t_net]
            elif isinstance(layer, NICECouplingLayer):
                nets += [layer.t_net]
    f = 0.0
    for net in nets:
        macs = [D.in_dim * D.out_dim for D in net]
        hidden = sum(macs[1:-1])
        fwd = sum(macs) if kernel_id == 6 else macs[0] + hidden
        f += 2.0 * (fwd + 2 * hidden)
    return f


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per GPU)
    with torch.distributed.run as a child process — before anything touches the
    GPU — and exit with its status.  Fails loudly when fewer than N devices are
    visible (a DF_DIST_BACKEND=gloo rehearsal may share devices)."""
    import socket
    import subprocess

    import torch

    backend = os.environ.get("DF_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()   # counts devices without initialising HIP
    if backend == "nccl" and ndev < args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus}: only {ndev} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, DF_BENCH_LAUNCHED="1")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU (default: the config's: 2^20 for cfg1/cfg2, 2^18 for cfg4 = configs[3] "
                         "and the per-GPU share of configs[4])")
    ap.add_argument("--mode", choices=["forward", "nll", "train"], default="forward")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="cfg2",
                    help="cfg2 is the headline (BASELINE configs[1]); cfg1/cfg4 are secondary measurements")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the exact-f32 FAST kernel timing that accompanies a SPLIT-kernel bench")
    ap.add_argument("--no-clock", action="store_true",
                    help="skip the clock run: a separate run of launches after the timed loop with the in-kernel "
                         "clock stamps on (df_chain_clock_probe); the timed launches never carry stamps")
    ap.add_argument("--settle-seconds", type=float, default=0.3,
                    help="untimed steps after the W warm-up steps until this much warm-up time has passed "
                         "(DVFS clock ramp; 0 = exactly W)")
    ap.add_argument("--graph", action="store_true",
                    help="train mode, one rank: replay each step as one hipGraph (df_train_step_graph)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous / timing plumbing only: no library, no GPU work (CPU tests)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    backend = os.environ.get("DF_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI
    if args.dry_run:
        if world > 1 and backend != "gloo":
            raise SystemExit("--dry-run with several ranks needs DF_DIST_BACKEND=gloo")
        return dry_run(args, world, rank)
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"WORLD_SIZE={world} ranks but only {ndev} GPU(s) visible")
    gpu = local % max(ndev, 1)          # ranks share a device only in gloo rehearsals
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist

        with _stdout_to_stderr():   # RCCL's init banner: stdout carries only the JSON line
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(backend)

    import densityflows_amd as dfa

    d, n, workload = CONFIGS[args.config]
    chain = build_chain(args.config)
    hc = chain.hip(device=gpu, n_hint=n)
    info = hc.info
    B = args.batch if args.batch is not None else (1 << 18 if args.config == "cfg4" else 1 << 20)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    zbuf = torch.randn(B * d, device=dev, generator=gen)      # Julia (d, B) column-major
    thbuf = torch.rand(B * n, device=dev, generator=gen) if n > 0 else None
    xbuf = torch.empty_like(zbuf)
    ldj = torch.empty(B, device=dev)
    s64 = torch.zeros(2, dtype=torch.float64, device=dev)

    trainer = None
    comm = None
    comm_error = None
    probe = hc                       # the handle whose chain-pass launches carry the clock stamps
    rehearsal = dist is not None and dist.get_backend() != "nccl"   # gloo: ranks may share one GPU
    if not rehearsal:
        # the library's own RCCL communicator (df_comm) carries every exchange of the
        # nll / train steps, at every rank count (world 1 included).  The forward step has
        # no exchange; there it only carries the per-rank report after the timed loop, and a
        # failure to build it is reported in the line instead of ending the run
        from densityflows_amd.parallel import DFComm

        try:
            with _stdout_to_stderr():
                comm = DFComm(gpu, rank, world)
        except Exception as e:          # noqa: BLE001
            if args.mode != "forward":
                raise
            comm_error = f"{type(e).__name__}: {e}"
    if args.mode == "forward":
        # the C-ABI call with its arguments bound once (the stream does not change): the
        # step is the library's host path + launch, not Python argument marshalling
        import ctypes as C
        from densityflows_amd.hip import _ptr, _stream
        fwd = hc.lib.df_chain_forward
        fwd_args = (hc.handle, _ptr(zbuf), _ptr(thbuf), _ptr(xbuf), _ptr(ldj), C.c_int64(B), _stream(dev))

        def step():
            rc = fwd(*fwd_args)
            if rc != 0:
                raise RuntimeError(hc.lib.df_last_error().decode())
    elif args.mode == "train":
        # one train! step (src/Flows.jl:398-413) on a fixed synthetic batch: inverse pass,
        # reverse sweep, gradient all-reduce across ranks (RCCL), Adam, weight repack
        from densityflows_amd.train import Adam, HIPTrainer

        hc.run("forward", zbuf, thbuf, xbuf, ldj, B)  # data points x = forward(z)
        trainer = HIPTrainer(hc, Adam(1e-3))

        def step():
            if args.graph and world == 1:
                trainer.step_graph(xbuf, thbuf, B, B, s64[:1])
                return
            if rehearsal:
                trainer.gradient(xbuf, thbuf, B, B * world, s64[:1])
                dist.all_reduce(trainer.grad())
                trainer.apply()
                return
            # gradient (global mean) → RCCL all-reduce of ∇ and Σ logpdf → Adam
            trainer.step_dist(comm, xbuf, thbuf, B, B * world, s64[:1])
    else:
        flow = dfa.Flow(chain, metadata=dfa.MetaData("", d, n, np.zeros(n, np.float32), np.ones(n, np.float32)))
        fh = flow.hip(device=gpu)
        probe = fh
        hc.run("forward", zbuf, thbuf, xbuf, ldj, B)  # data points x = forward(z)

        nll = fh.lib.df_flow_nll
        import ctypes as C
        from densityflows_amd.hip import _ptr, _stream
        nll_args = (fh.handle, comm.handle if comm is not None else None, _ptr(xbuf), _ptr(thbuf), C.c_int64(B), C.c_void_p(s64.data_ptr()),
                    _stream(dev))

        def step():
            # fused inverse + logpdf + fp64 Σ of this rank's shard, {Σ, N} all-reduced over RCCL (df_flow_nll)
            rc = nll(*nll_args)
            if rc != 0:
                raise RuntimeError(fh.lib.df_last_error().decode())
            if rehearsal:
                dist.all_reduce(s64)

    stream = torch.cuda.current_stream(dev)
    steplog = os.environ.get("DF_BENCH_STEPLOG") == "1"   # diagnostic: per-step HIP-event times on stderr
    warm_ms = []
    t_warm = time.perf_counter()
    for _ in range(args.warmup):
        if steplog:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            step()
            e1.record(stream)
            warm_ms.append((e0, e1))
        else:
            step()
    torch.cuda.synchronize()
    # clock settle: the chip ramps its shader clock over the first ~50 ms of back-to-back
    # launches (profiles/r03_clock_ramp.txt: 2.00 GHz over steps 6-25, 2.25 GHz after 50);
    # untimed steps continue until --settle-seconds of warm-up have passed, so the K timed
    # steps measure the steady state whatever W is (reported as clock_settle)
    settle_steps, t_w = 0, time.perf_counter()
    while time.perf_counter() - t_warm < args.settle_seconds and settle_steps < 100000:
        for _ in range(8):
            step()
        settle_steps += 8
        torch.cuda.synchronize()
    settle_s = time.perf_counter() - t_w
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if steplog else None
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        if steplog:
            step_ev[i].record(stream)
        step()
    if steplog:
        step_ev[-1].record(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)                 # HIP events on the launch stream
    clock = None
    if not args.no_clock:
        # the clock run: the same steps right after the timed loop (the chip still at its
        # steady clock) with the in-kernel stamps on; the timed launches above ran the plain
        # production kernels
        k_clk = min(max(args.steps, 1), 50)
        probe.clock_probe(True)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for _ in range(k_clk):
            step()
        c1.record(stream)
        torch.cuda.synchronize()
        clk_ms = c0.elapsed_time(c1) / k_clk
        ghz_med, ghz_mean, slots = probe.clock_read()
        probe.clock_probe(False)
        if slots > 0:
            clock = {"ghz_median": round(ghz_med, 4), "ghz_sum_ratio": round(ghz_mean, 4), "workgroup_slots": slots,
                     "kernel_mcycles_per_launch": None, "clock_run_steps": k_clk,
                     "clock_run_ms_per_step": round(clk_ms, 4),
                     "source": "in-kernel s_memtime / s_memrealtime (100 MHz) stamps by wave 0 of every workgroup, "
                               "taken in a separate run of clock_run_steps launches right after the timed loop "
                               "(df_chain_clock_probe); the timed launches carry no stamps"}
    if steplog:
        print(json.dumps({"rank": rank, "warmup_ms": [round(a.elapsed_time(b), 4) for a, b in warm_ms],
                          "step_ms": [round(step_ev[i].elapsed_time(step_ev[i + 1]), 4) for i in range(args.steps)]}),
              file=sys.stderr, flush=True)
    elapsed = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    ranks = rank_report(dist, dev, gpu_ms / args.steps, wall * 1e3 / args.steps, world, B, comm, comm_error,
                        "torch.distributed " + (dist.get_backend() if dist is not None else "none"))
    total = B * world * args.steps
    value = total / elapsed / 1e6
    kernel_s = gpu_ms / 1e3 / args.steps            # mean launch time (one launch per step)
    if clock is not None and args.mode != "train":
        # clock-normalised time: shader cycles per launch of the clock run (comparable across
        # boxes and DVFS states)
        clock["kernel_mcycles_per_launch"] = round(clock["clock_run_ms_per_step"] * clock["ghz_median"], 4)
    flop = info.flops_per_sample * B
    achieved_tflops = flop / kernel_s / 1e12
    hbm_algo = (8.0 * d + 4.0 * n + 4.0) * B          # read z (+θ), write x, ldj

    # roofline peak of the arithmetic the kernels run: the SPLIT kernels compute their
    # GEMMs on bf16 MFMA (six products per f32 product), the rest on f32 MFMA / VALU
    kernel_id = int(getattr(info, "kernel", 3))
    f_all = float(info.flops_per_sample)
    f_split = float(getattr(info, "split_flops_per_sample", 0.0))
    if args.mode == "train":
        # algorithmic training work: forward + 2× backward (dX and dW) = 3F per sample
        f_all = 3.0 * f_all
        f_split = train_split_flops(chain, kernel_id)
        achieved_tflops = f_all * B / kernel_s / 1e12
    peak = PEAK_F32_TFLOPS
    if f_split > 0.0:
        peak = f_all / (f_split / PEAK_SPLIT_TFLOPS + (f_all - f_split) / PEAK_F32_TFLOPS)

    exact = None
    if kernel_id in (4, 6) and args.mode == "forward" and not args.no_exact:
        # the same launches on the exact-f32 kernel: a second handle planned under
        # DF_F32_EXACT=1 (a chain's arithmetic is fixed when it is created)
        from densityflows_amd.hip import HIPChain

        os.environ["DF_F32_EXACT"] = "1"
        hx = HIPChain(chain.layers, device=gpu, n_hint=n)
        del os.environ["DF_F32_EXACT"]

        def step():
            hx.run("forward", zbuf, thbuf, xbuf, ldj, B)

        for _ in range(min(args.warmup, 20)):
            step()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k_exact = max(20, args.steps // 4)
        e0.record(stream)
        for _ in range(k_exact):
            step()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k_exact
        exact = {"kernel": KERNELS[kernel_id - 1], "ms_per_step": round(ms, 4), "value": round(B * world / ms / 1e3, 3),
                 "frac_of_f32_peak": round(f_all * B / (ms / 1e3) / 1e12 / PEAK_F32_TFLOPS, 4), "steps": k_exact}

    traffic, traffic_src, pmc = None, None, {}
    default_b = (1 << 18) if args.config == "cfg4" else (1 << 20)
    if args.config in TRAFFIC_PROFILES and args.mode == "forward" and B == default_b:
        traffic_src = TRAFFIC_PROFILES[args.config]
        pmc = pmc_summary(traffic_src)
        traffic = pmc["traffic"]
    if rank == 0:
        out = {
            "metric": {"forward": METRIC, "nll": "NLL (inverse+logpdf+Σ, RCCL all-reduce) Msamples/s",
                       "train": "train! step (inverse+NLL+backward+Adam, RCCL gradient all-reduce) Msamples/s"
                       }[args.mode],
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",   # f32 in / f32 out at f32-level error; kernel arithmetic in roofline.kernel
            "data": "synthetic: z ~ N(0,1) generated on device; random-init weights (glorot, see bench.build_chain)",
            "config": {"workload": workload + ("" if world == 1 else f"; config3 sharding {world}x"),
                       "per_gpu_batch": B, "global_batch": B * world,
                       "parallelism": {"forward": f"dp{world} (independent sample shards, no data-path collective)",
                                       "nll": f"dp{world} + RCCL all-reduce of the NLL partial",
                                       "train": f"dp{world} + RCCL all-reduce of the flat gradient"}[args.mode]},
            "roofline": {"bound": "mfma", "achieved": round(achieved_tflops, 3), "peak": round(peak, 2),
                         "unit": "TFLOP/s", "frac": round(achieved_tflops / peak, 4),
                         "kernel": KERNELS.get(kernel_id, str(kernel_id)),
                         "peak_basis": ("f32 MFMA 157.3 TF" if f_split == 0.0 else
                                        f"mix: {f_split:.0f} of {f_all:.0f} FLOP/sample at the bf16x3 split rate "
                                        f"{PEAK_SPLIT_TFLOPS:.1f} TF (bf16 MFMA / 6), the rest at f32 157.3 TF"),
                         "frac_of_f32_mfma_peak": round(achieved_tflops / PEAK_F32_TFLOPS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src if traffic is not None else None,
                         "mfma_busy": pmc.get("mfma_busy"),
                         "pmc_source_sha16": pmc.get("source"),
                         "pmc_matches_benched_source": (pmc.get("source") == source_sha16())
                         if pmc.get("source") else None,
                         "kernel_ms": round(kernel_s * 1e3, 4),
                         "kernel_ms_scope": "whole step (all launches)" if args.mode == "train" else "one launch",
                         "algorithmic_flop_per_sample": f_all,
                         "hbm_algorithmic_GBps": round(hbm_algo / kernel_s / 1e9, 2)},
            "clock": clock,
            "clock_settle": {"untimed_steps_after_warmup": settle_steps, "seconds": round(settle_s, 3),
                             "target_seconds_of_warmup": args.settle_seconds,
                             "policy": "after the W warm-up steps, untimed steps run until settle-seconds of "
                                       "warm-up have passed (DVFS clock ramp); the K timed steps are unchanged"},
            "ranks": ranks,
        }
        if args.mode == "train" and clock is not None:
            clock["scope"] = "the inverse chain pass of each step only"
        if args.config != "cfg2":
            out["metric"] = out["metric"].replace("d=5 8-layer RealNVP", CONFIGS[args.config][2].split(":")[0])
        if exact is not None:
            out["f32_exact_kernel"] = exact
        if world == 1 and not args.no_cpu and args.mode == "forward":
            # config 1 is the reference's CPU case at B = 4096 (BASELINE configs[0])
            out["cpu_baseline"] = cpu_baseline(chain, d, n, seconds=args.cpu_seconds,
                                               sample=4096 if args.config == "cfg1" else 65536)
            out["vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if args.mode == "nll" and rank == 0:
        loss = -float(s64[0].item()) / float(s64[1].item())
        assert s64[1].item() == B * world and np.isfinite(loss), "df_flow_nll returned an inconsistent {Σ, N}"
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


def rank_report(dist, dev, kernel_ms, wall_ms, world, batch, comm, comm_error, group_desc):
    """Per-rank timing spread and the communicator behind the line:
    every rank's mean kernel (HIP-event) and wall time per step, gathered to rank 0
    (min / max / per rank); the df_comm size from df_comm_get_info, and one RCCL
    all-reduce of this rank's sample count through it, checked against B x world.
    Runs after the timed loop."""
    import torch

    mine = torch.tensor([kernel_ms, wall_ms], dtype=torch.float64, device=dev)
    if dist is not None:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        allv = torch.stack(allv).cpu().tolist()
    else:
        allv = [mine.cpu().tolist()]
    k = [v[0] for v in allv]
    w = [v[1] for v in allv]
    out = {"n": len(allv), "kernel_ms_min": round(min(k), 4), "kernel_ms_max": round(max(k), 4),
           "wall_ms_per_step_min": round(min(w), 4), "wall_ms_per_step_max": round(max(w), 4),
           "kernel_ms_per_rank": [round(x, 4) for x in k], "process_group": group_desc, "df_comm": None}
    if comm is not None:
        r, nr, d = comm.info()
        cnt = torch.tensor([float(batch), float(nr)], dtype=torch.float64, device=dev)
        comm.allreduce_(cnt)
        torch.cuda.synchronize()
        out["df_comm"] = {"nranks": nr, "rank": r, "device": d,
                          "allreduce_count_ok": float(cnt[0].item()) == float(batch) * world,
                          "allreduce_nranks_sum": float(cnt[1].item())}
    elif comm_error is not None:
        out["df_comm"] = {"error": comm_error}
    return out


def dry_run(args, world, rank):
    """The bench's launch, rendezvous and max-over-ranks timing without the
    library or a GPU: tests of `--gpus N` self-launching run it on CPU (gloo)."""
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        pass
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    elapsed = torch.tensor([wall], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    ranks = rank_report(dist, torch.device("cpu"), 0.0, wall * 1e3 / max(args.steps, 1), world, 0, None, None,
                        "torch.distributed " + (dist.get_backend() if dist is not None else "none"))
    ranks["group_size"] = dist.get_world_size() if dist is not None else 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Msamples/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                          "ms_per_step": float(elapsed.item()) * 1e3 / max(args.steps, 1), "ranks": ranks}),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
