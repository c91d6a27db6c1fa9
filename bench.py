"""Headline benchmark: env-steps/s of the batched assignment-env rollout on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 0..4] [--selector eps|sap|random]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

--config i selects BASELINE.json configs[i] (default 2; 3 is configs[2] per GPU on N GPUs):
  0  4 x 4, 1 env, fused RNN agent + epsilon-greedy  (the reference's CPU plumbing case)
  1  16 x 16, 4,096 envs per GPU, random policy
  2  64 x 64, 16,384 envs per GPU, BasicMAC + RNNAgent (GRU 64, fp32) + epsilon-greedy 0.05
  3  as 2 on every rank of an N-GPU job (131,072 envs at N = 8; weak scaling)
  4  256 x 256 dense benefits, 2,048 envs per GPU, BasicMAC + RNNAgent + epsilon-greedy
Explicit --n/--m/--envs/--selector/--agent/--benefits override the config's values.

One "step" = one transition of every env on every rank plus the action selection of the
next row (agent forward + selector, writing the EpisodeBatch).  Default schedule (the
runner's, args.fused_rollout): asg_reset, then the whole episode -- selection on the reset
row, T transitions, the selections in between -- in ONE asg_rollout launch of the fused
rollout kernel (env transition + RNNAgent forward + epsilon-greedy, csrc/asg_h2.hip); the
timed window's edges cut episodes into chunks (select_first / select_last at the seams).
--fused-rollout 3 times one launch per step, 0 the separate env-step and agent kernels.
Every T steps an episode ends (returns all-gathered on the device) and the next one is
reset inside the timed region; the host-side episode checks (device error words, selector
status, logging) run once after it (GpuVecRunner.finish_episode(sync=False) /
flush_pending).  value = (sum over ranks of envs) * K / (max over ranks of the K-step time).

The JSON line also carries:
  roofline        the dominant kernel: the fused rollout kernel (algorithmic bytes per step
                  B_step + n (2*4*64 + 8) per env, DESIGN.md §3, over its mean HIP-event time per
                  step on the stream it is launched on) against 8 TB/s; `traffic` = PMC HBM bytes
                  (profiles/*pmc_rollout_kernel*.json), `issue` = its SQ figures, `bound` derived
                  from them (HBM or the store-ordered latency).  On the split schedule: the env
                  step kernel (SURVEY §8(d)'s B_step * E).
  roofline_agent  the agent kernel (split-schedule leg) against its MFMA roof and HBM.
  kernels_ms      per-step kernel times (fused rollout / env step / selection).
  cpu_baseline    rank 0 at N = 1 only: the reference's CPU design (subprocess-per-env
                  ParallelRunner + numpy env + CPU RNN agent, oracle/cpu_parallel_runner.py) on
                  a bounded sample of the same workload: step-loop-only and reset-amortised
                  rates, the worker count used and the host's core count.
  secondary       (N = 1, --secondary 1, the default then; each leg with its own value and
                  ms_per_step): split_rollout (separate launches), step_rollout (one fused
                  launch per step), pytorch_agent (configs[2] read literally: the PyTorch
                  RNNAgent + asg_epsilon_greedy), sap (fused noise + LSA per env, roofline_lsa
                  against both issue bounds), iql / reda (the reference's mock algorithms:
                  jumpstart_mac + HAA jumpstart, Linear agent, eps-greedy / SAP), config4
                  (BASELINE configs[4]: 256 x 256 dense, 2,048 envs, fused rollout).
"""
import argparse
import gc
import glob
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFS = 157.3  # MI355X dense f32 MFMA (= f32 vector peak; MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md)
# f32 products as three-way-split bf16 MFMAs cost six bf16 products each
X3_PEAK_TFS = BF16_MFMA_PEAK_TFS / 6
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs, max clock (MI355X_MICROARCH.md)
VALU_CYCLES_PER_WAVE_INSTR = 2  # wave64 VALU over a SIMD-32 (MI355X_MICROARCH.md "Wave scheduling")
FUSED_AGENTS = ("rnn", "rnn_fused")  # agent names that resolve to RNNFusedAgent (modules/agents)
CPU_WORKER_CAP = 16  # CPU share of one GPU on the gpurun box (os.cpu_count() shows the whole host)

CONFIGS = {
    0: dict(n=4, m=4, envs=1, selector="eps", agent="rnn", benefits="bump",
            label="4-agent/4-task assignment env, batch_size_run=1 (configs[0]: the reference's plumbing case)"),
    1: dict(n=16, m=16, envs=4096, selector="random", agent="rnn", benefits="bump",
            label="16-agent/16-task assignment env, 4096 envs per GPU, random policy (configs[1])"),
    2: dict(n=64, m=64, envs=16384, selector="eps", agent="rnn", benefits="bump",
            label="64-agent/64-task assignment env, 16384 envs per GPU, BasicMAC+RNN (configs[2])"),
    3: dict(n=64, m=64, envs=16384, selector="eps", agent="rnn", benefits="bump",
            label="64-agent/64-task assignment env, 16384 envs per GPU sharded over the node (configs[3])"),
    4: dict(n=256, m=256, envs=2048, selector="eps", agent="rnn", benefits="dense",
            label="256-agent/256-task dense-benefit assignment env, 2048 envs per GPU (configs[4])"),
}


def step_bytes(n, m, L):
    """Algorithmic HBM bytes of one env step: obs f32 n*m*(L+1),
    beta f32 n*m, avail_actions bool n*m, actions_onehot i64 n*m, actions i64 n (read),
    rewards f32 n, prev_assigns i64 n, terminated 1 B, filled 8 B."""
    return n * m * (4 * (L + 1) + 4 + 1 + 8) + n * (8 + 4 + 8) + 1 + 8


F16_MFMA_PEAK_TFS = 2500.0  # dense f16 MFMA = bf16 rate (MI355X_MICROARCH.md)
# f32 products as two-way-split f16 MFMAs cost three f16 products each
H2_PEAK_TFS = F16_MFMA_PEAK_TFS / 3


def agent_peak(n, m, L, mode, hidden=64, use_rnn=True, onehot=True):
    """f32-equivalent MFMA roof of the agent forward: each layer's flops at the peak of the
    MFMA it runs on (asg_rnn_agent_mode: 4 = every layer on split f16; else bit 0 GRU, bit 1
    fc1 on split bf16), combined as the time-weighted harmonic mean (flops / sum of
    per-layer minimum times)."""
    if mode == 4:
        return H2_PEAK_TFS
    K = m * (L + 1) - (m if onehot else 0)
    fc1, rec, fc2 = 2 * K * hidden, 2 * (2 * 3 * hidden * hidden if use_rnn else hidden * hidden), 2 * hidden * m
    t = (fc1 / (X3_PEAK_TFS if mode & 2 else F32_MFMA_PEAK_TFS) + rec / (X3_PEAK_TFS if mode & 1 else F32_MFMA_PEAK_TFS)
         + fc2 / F32_MFMA_PEAK_TFS)
    return (fc1 + rec + fc2) / t


def agent_flops(n, m, L, hidden=64, use_rnn=True, onehot=True):
    """Algorithmic flops of one agent row: fc1 (m(L+1) -> hidden), GRUCell (two hidden x
    3*hidden products), fc2 (hidden -> m); 2 flops per multiply-add.  onehot: the obs
    one-hot block (the first m inputs) is a column gather of W1, not m*hidden products
    (the fused kernel's one-hot prefix; a -DASG_AGENT_ONEHOT=0 build turns it off), so fc1
    counts K - m inputs."""
    K = m * (L + 1) - (m if onehot else 0)
    rec = 2 * 3 * hidden * hidden if use_rnn else hidden * hidden
    return 2 * (K * hidden + rec + hidden * m)


def agent_bytes(n, m, L, hidden=64):
    """Algorithmic HBM bytes of one agent row of the fused forward + selection: the obs row
    (f32 m(L+1)), h in and h' out (f32 hidden each), the availability row (bool m) and the
    int64 action written."""
    return 4 * m * (L + 1) + 2 * 4 * hidden + m + 8


def agent_roofline(a, E, agent_ms, kernel):
    """The agent forward (timed with HIP events on its stream) against its MFMA roof and
    against HBM (both reported; `bound` names the larger fraction)."""
    if agent_ms is None or agent_ms <= 0:
        return None
    fused = a.agent in FUSED_AGENTS
    onehot = fused
    flops = agent_flops(a.n, a.m, a.L, onehot=onehot) * E * a.n
    tfs = flops / (agent_ms * 1e-3) / 1e12
    from marl_sap_amd import _lib
    K = a.m * (a.L + 1)
    mode = int(_lib.lib().asg_rnn_agent_mode(K, 64, a.m, 1)) if fused else 0
    peak = agent_peak(a.n, a.m, a.L, mode, onehot=onehot)
    nbytes = agent_bytes(a.n, a.m, a.L) * E * a.n
    gbs = nbytes / (agent_ms * 1e-3) / 1e9
    mfma = {"achieved": round(tfs, 2), "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(tfs / peak, 4),
            "peak_note": {4: "f32-equivalent: every layer's products on two-way-split f16 MFMAs (2.5 PF / 3)",
                          0: "f32 MFMA peak"}.get(mode, "f32-equivalent: GRU products on three-way-split bf16 "
                                                        "MFMAs (2.5 PF / 6), fc1/fc2 on f32 MFMAs (157.3 TF), "
                                                        "time-weighted")}
    hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
           "bytes_per_launch": nbytes}
    # PMC HBM bytes of the same kernel at this workload (FETCH_SIZE doubled for its 16-B/lane
    # streaming reads, + WRITE_SIZE; tools/pmc_summary.py), when profiled
    pm = pmc_lookup("*pmc_agent_hbm*.json", n=a.n, m=a.m, E=E) if fused else None
    traffic = None
    if pm and pm.get("kernel") in pm.get("kernels", {}):
        traffic = round(pm["kernels"][pm["kernel"]]["hbm_bytes_fetch_doubled"])
        hbm["traffic"] = traffic
    top = hbm if hbm["frac"] >= mfma["frac"] else mfma
    return {"bound": "hbm" if top is hbm else "mfma", "achieved": top["achieved"], "peak": top["peak"],
            "unit": top["unit"], "frac": top["frac"], "traffic": traffic if top is hbm else None, "mfma": mfma,
            "hbm": hbm,
            "kernel": kernel, "kernel_ms": round(agent_ms, 4), "flops_per_launch": flops}


def profile_order(path):
    """Sort key of a profiles/ file: (round, session, name).  Files are named
    r<round>_<what>_s<session>[suffix].json; the round-1 files carry neither (round 1,
    session 0).  Numeric, so r3_..._s10 sorts after r3_..._s9."""
    import re
    name = os.path.basename(path)
    mr = re.match(r"r(\d+)_", name)
    ms = re.search(r"_s(\d+)[a-z]?\.[a-z]+$", name)
    return (int(mr.group(1)) if mr else 1, int(ms.group(1)) if ms else 0, name)


def pmc_lookup(pattern, **match):
    """Newest profiles/ summary matching the workload keys (n, m, E, L), else None."""
    # newest first by (round, session) parsed from the name (profile_order)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=profile_order, reverse=True):
        try:
            pm = json.load(open(path))
        except (ValueError, OSError):
            continue
        if all(pm.get(k) == v for k, v in match.items()):
            pm["_path"] = path
            return pm
    return None


def reset_bytes(n, m, L):
    """Algorithmic HBM bytes of one env's reset (asg_reset): the pre-transition row (obs f32
    n*m*(L+1), beta f32 n*m, avail n*m) plus prev_assigns i64 n and filled 8 B."""
    return n * m * (4 * (L + 1) + 4 + 1) + 8 * n + 8


def store_ceiling(hbm=True):
    """The measured store ceiling (GB/s): the best shape of the newest tools/store_bw.hip record
    under profiles/, with the file name.  hbm=True: store-only streams over a buffer far larger
    than the 256 MiB MALL (the HBM write ceiling); False: the `reuse` shape (one 256 MiB buffer
    rewritten in a loop, the REDA Q buffer's pattern -- a MALL rate, not an HBM one)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*store_bw*.txt")), key=profile_order, reverse=True)
    for f in files:
        best = 0.0
        for line in open(f):
            if line.startswith("{"):
                try:
                    d = json.loads(line)
                    if bool(d.get("hbm", d.get("shape") != "reuse")) == hbm:
                        best = max(best, float(d["GBps"]))
                except (ValueError, KeyError):
                    pass
        if best > 0:
            return best, os.path.basename(f)
    return None, None


def fused_roofline(a, E, fused_ms, use_rnn=True, resets_per_step=0.0, q_out=False, bids=False):
    """Roofline of the fused rollout kernel (asg_rollout -> rollout_kernel), per env step: the
    env step's bytes plus the agent's h in / h out and the action written -- the observations
    it generates are consumed on chip, never read back -- per env, times E, over its HIP-event
    time per step (a launch of s steps counts s).  Linear agent (use_rnn False): no h read.
    `frac` is against HBM; `bound` names what binds, from the kernel's SQ counters when
    profiled (tools/round_profile.sh): "latency/store-ack" when neither VALU issue nor the
    MFMA pipe is at half its capacity and HBM is not near its roof (the waves wait on the
    in-order vmcnt queue behind their own row stores).  q_out: the
    asg_step_forward instances (REDA's step_q schedule), which also write the Q rows (4 m per
    agent) and read the actions row the SAP kernel wrote instead of writing one.  bids: the
    bids_as_actions env (no actions_onehot field; the transition reads the int32 assignments
    asg_bids_select left instead of the int64 actions row); no PMC profile of it is kept."""
    # the episode's reset runs in its first launch (asg_reset_rollout): its row counts too.
    # q_out: the Q rows go to ONE reused [E n][m] f32 buffer (basic_controller._q_buf, 256 MiB at
    # configs[2] = the MALL's size) rewritten every step and read back by the SAP kernel: much of
    # it stays in the Infinity Cache, so its bytes are reported apart (q_buffer), not as HBM traffic
    sb = step_bytes(a.n, a.m, a.L) - (8 * a.n * a.m + 4 * a.n if bids else 0)
    per_launch = (sb + a.n * ((2 if use_rnn else 1) * 4 * 64 + 8)
                  + resets_per_step * reset_bytes(a.n, a.m, a.L)) * E
    q_bytes = 4 * a.n * a.m * E if q_out else 0
    per_launch = int(round(per_launch))
    achieved = per_launch / (fused_ms * 1e-3) / 1e9
    frac = achieved / HBM_PEAK_GBS
    tag = "rollout_q" if q_out else "rollout"
    pm = None if bids else pmc_lookup(f"*pmc_{tag}_kernel*.json", n=a.n, m=a.m, E=E, L=a.L, use_rnn=bool(use_rnn))
    issue = None
    pq = None if bids else pmc_lookup(f"*pmc_{tag}_sq*.json", n=a.n, m=a.m, E=E, L=a.L, use_rnn=bool(use_rnn))
    if pq:
        c, d = pq["counters"], pq["derived"]
        spl = pq.get("steps_per_launch", 1)  # the profiled launches ran spl steps each
        issue = {"valu_insts_per_step": round(c["SQ_INSTS_VALU"] / spl),
                 "mfma_insts_per_step": round(c["SQ_INSTS_MFMA"] / spl),
                 "valu_issue_frac": round(c["SQ_INSTS_VALU"] / spl * VALU_CYCLES_PER_WAVE_INSTR
                                          / (SIMDS * CLOCK_HZ * fused_ms * 1e-3), 4),
                 "mfma_busy_frac": round(d["mfma_busy_frac"], 4), "wait_any_frac": round(d["wait_any_frac"], 4),
                 "pmc": os.path.basename(pq.get("_path", "")) or None}
    bound = "hbm"
    if issue and issue["valu_issue_frac"] < 0.5 and issue["mfma_busy_frac"] < 0.5 and frac < 0.6:
        bound = "latency/store-ack"
    traffic = None
    if pm:
        # the profiled launch is one whole episode: its reset row + steps_per_launch steps
        # (resets_per_launch, 1 for tools/round_profile.sh's launches).  Put the reset on the
        # same side as bytes_per_launch: per step, the profile's reset share is replaced by
        # this window's (resets_per_step) at the reset's algorithmic size, so that
        # traffic / bytes_per_launch is the measured-over-algorithmic ratio of the steps
        spl = pm.get("steps_per_launch", 1)
        rpl = pm.get("resets_per_launch", 1 if spl > 1 else 0)
        rb = reset_bytes(a.n, a.m, a.L) * E
        traffic = round((pm["hbm_bytes_per_launch"] - rpl * rb) / spl + resets_per_step * rb)
        if q_out:
            traffic = None  # the PMC bytes mix the Q buffer's MALL-resident writes with HBM
    out = {"bound": bound, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(frac, 4),
           "traffic": traffic,
           "kernel": ("asg::rollout_kernel Q-output instance (asg_step_forward: env step + agent forward)" if q_out
                      else "asg::rollout_kernel (env steps + agent/eps-greedy selections, per step)"),
           "kernel_ms": round(fused_ms, 4), "bytes_per_launch": per_launch,
           "per_launch_note": "per env step of the launch (bytes_per_launch, kernel_ms: one step's share; "
                              "the fused resets' rows amortised over the timed steps)",
           "resets_per_step": round(resets_per_step, 4),
           "frac_note": "frac is against the 8 TB/s HBM peak"}
    # the kernel writes almost all of its bytes: against the measured store ceiling too (writes
    # = the rows, h out, the action, Q; reads = h in)
    ceil, ceil_src = store_ceiling()
    if ceil:
        reads = (a.n * 4 * 64 if use_rnn else 0) * E
        writes = per_launch - reads - 8 * a.n * E  # B_step counts the actions row as a read: it stays in LDS
        wgbs = writes / (fused_ms * 1e-3) / 1e9
        out["store_ceiling"] = {"write_bytes_per_launch": int(writes), "achieved_write_GBps": round(wgbs, 1),
                                "ceiling_GBps": ceil, "frac": round(wgbs / ceil, 4), "source": ceil_src,
                                "note": "the batch rows' writes (the Q buffer excluded) against the HBM store-only "
                                        "ceiling measured by tools/store_bw.hip on MI355X (streams over a buffer far "
                                        "larger than the MALL)"}
    if q_out:
        qc, _ = store_ceiling(hbm=False)
        out["q_buffer"] = {"bytes_per_launch": q_bytes, "GBps_if_alone": round(q_bytes / (fused_ms * 1e-3) / 1e9, 1),
                           "reuse_store_GBps": qc,
                           "note": "Q rows [E n][m] f32 written to one reused 256 MiB buffer every step (read back by "
                                   "the SAP kernel): MALL-resident in large part, so not counted in bytes_per_launch / "
                                   "frac / store_ceiling; reuse_store_GBps = tools/store_bw.hip's 'reuse' shape"}
    if pm and traffic:
        out["traffic_pmc"] = os.path.basename(pm.get("_path", ""))
        out["traffic_over_algorithmic"] = round(traffic / per_launch, 4)
        out["traffic_note"] = ("PMC bytes per step of the profiled whole-episode launch, its reset row's share "
                               "replaced by this window's resets_per_step (same accounting as bytes_per_launch)")
    if issue:
        out["issue"] = issue
    # SURVEY §8(d)'s own accounting beside the one above: B_batch = B_env + the fused int64 one-hot
    # (8nm) + the actions written (8n) per env-step, + the reset row per reset -- no hidden state
    # (the agent's h round trip is design traffic of this kernel, not the path's)
    b_env = a.n * a.m * (4 * a.L + 13) + 20 * a.n + 9
    b_batch = int(round((b_env + 8 * a.n * a.m + 8 * a.n + resets_per_step * reset_bytes(a.n, a.m, a.L)) * E))
    sv = b_batch / (fused_ms * 1e-3) / 1e9
    out["survey_b_batch"] = {"bytes_per_launch": b_batch, "achieved": round(sv, 1), "frac": round(sv / HBM_PEAK_GBS, 4),
                             "note": "SURVEY §8(d) B_batch = nm(4L+13) + 20n + 9 + 8nm + 8n per env-step (+ the reset "
                                     "row amortised), against the 8 TB/s peak"}
    return out


def random_roofline(a, E, ms, resets_per_step):
    """The random policy's episode kernel (asg_random_rollout -> random_rollout_kernel), per env
    step: B_step (the actions row written instead of read) plus the reset row per env for each
    reset in the window, over its HIP-event time per step."""
    per_launch = int(round((step_bytes(a.n, a.m, a.L) + resets_per_step * reset_bytes(a.n, a.m, a.L)) * E))
    achieved = per_launch / (ms * 1e-3) / 1e9
    pm = pmc_lookup("*pmc_random_rollout*.json", n=a.n, m=a.m, E=E, L=a.L)
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "kernel": "asg::random_rollout_kernel (uniform actions + transition, per step)",
           "kernel_ms": round(ms, 4), "bytes_per_launch": per_launch, "resets_per_step": round(resets_per_step, 4),
           "b_env_survey_per_launch": (a.n * a.m * (4 * a.L + 13) + 20 * a.n + 9) * E,
           "per_launch_note": "per env step of the launch: B_step = SURVEY §8(d)'s B_env + the fused int64 one-hot "
                              "(8nm) - the table read (bumps regenerated, 4nm), + the reset row amortised"}
    if pm:
        spl = pm.get("steps_per_launch", 1)
        rpl = pm.get("resets_per_launch", 1)
        rb = reset_bytes(a.n, a.m, a.L) * E
        out["traffic"] = round((pm["hbm_bytes_per_launch"] - rpl * rb) / spl + resets_per_step * rb)
        out["traffic_pmc"] = os.path.basename(pm.get("_path", ""))
    return out


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    p.add_argument("--envs", type=int, default=None, help="envs per GPU")
    p.add_argument("--n", type=int, default=None)
    p.add_argument("--m", type=int, default=None)
    p.add_argument("--T", type=int, default=20)
    p.add_argument("--L", type=int, default=3)
    p.add_argument("--selector", default=None, choices=["eps", "sap", "random", "bids"])
    p.add_argument("--benefits", default=None, choices=["bump", "dense"])
    p.add_argument("--rng", default="philox", choices=["philox", "mt19937"],
                   help="mt19937: the same-seed mode (env e replays numpy's legacy stream seeded with seed + e; "
                        "float32 benefit table + recorded draws)")
    p.add_argument("--agent", default=None, choices=["rnn", "rnn_fused", "rnn_torch"],
                   help="rnn (the reference's name; default): the RNNAgent with its inference forward as one HIP "
                        "kernel wherever the shape allows (= rnn_fused); rnn_torch: the plain PyTorch module")
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-episodes", type=int, default=2, help="minimum CPU-baseline episodes")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample length (s)")
    p.add_argument("--cpu-workers", type=int, default=None,
                   help=f"CPU-baseline env workers (default min(os.cpu_count(), {CPU_WORKER_CAP}))")
    p.add_argument("--secondary", type=int, default=-1, help="secondary legs (-1: on at N = 1 for configs 2/3)")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--fused-rollout", type=int, default=1, choices=[0, 1, 2, 3],
                   help="1 (default): the whole episode -- env steps + agent/eps-greedy selections -- in one kernel "
                        "(asg_rollout); 3: one asg_rollout launch per step (env step t + selection t + 1); 0: separate "
                        "asg_step + agent select launches; 2: as 1")
    p.add_argument("--use-rnn", type=int, default=1, help="0: the Linear + ReLU RNNAgent (use_rnn: False)")
    p.add_argument("--sap-warm", type=int, default=1,
                   help="1 (default): the SAP selector's fast path warm-started from the previous step's duals")
    p.add_argument("--real-envs", type=int, default=512,
                   help="envs of the secondary real-env leg (324 x 450, T = 100; ~280 MB of tables + batch per env); "
                        "0: skip it")
    p.add_argument("--fuse-reset", type=int, default=1,
                   help="1 (default, the runner's): on the episode schedule the env reset runs in the episode's "
                        "first launch (asg_reset_rollout); 0: asg_reset as its own launch")
    a = p.parse_args(argv)
    cfg = CONFIGS[a.config]
    for k in ("n", "m", "envs", "selector", "agent", "benefits"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    return a


def make_args(a, E, selector=None, agent=None, fused=None, mac="basic_mac", use_rnn=None, **extra):
    selector = selector or a.selector
    fused = a.fused_rollout if fused is None else fused
    sel = {"eps": "epsilon_greedy", "sap": "sap", "random": "epsilon_greedy", "bids": "continuous"}[selector]
    args = SimpleNamespace(
        batch_size_run=E, env="mock_constellation_env",
        env_args=dict(n=a.n, m=a.m, T=a.T, L=a.L, lambda_=0.5, bids_as_actions=False, seed=a.seed,
                      benefits=a.benefits),
        env_rng=a.rng, env_quirks=(), runner_protocol="episode", test_nepisode=1,
        runner_log_interval=10 ** 12, n=a.n, m=a.m, T=a.T, hidden_dim=64,
        use_rnn=bool(a.use_rnn if use_rnn is None else use_rnn),
        obs_last_action=False, obs_agent_id=False, agent_output_type="q", action_selector=sel,
        agent=agent or a.agent, seed=a.seed,
        epsilon_start=0.05, epsilon_finish=0.05, epsilon_anneal_time=1, evaluation_epsilon=0.0, mac=mac,
        reuse_batch=True, fused_rollout={0: False, 1: True, 2: "always", 3: "step"}[fused],
        sap_warm_start=bool(a.sap_warm))
    if selector == "bids":
        # config/algs/ippo_sap.yaml's env path: bids_as_actions, the continuous selector over
        # softmaxed pi_logits (use_rnn False), its epsilon 0.3 -> 0.05 over 50,000 env steps
        args.env_args["bids_as_actions"] = True
        args.agent_output_type, args.softmax_agent_inputs, args.use_rnn = "pi_logits", True, False
        args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time = 0.3, 0.05, 50000
    for k, v in extra.items():
        setattr(args, k, v)
    return args


class NullLogger:
    def log_stat(self, *a, **k):
        pass


def cpu_baseline(a):
    """The reference's CPU design on this host (oracle/cpu_parallel_runner.py), SURVEY §8(d):
    one worker process per env, batch_size_run = os.cpu_count() capped at the GPU's CPU
    share; rates with resets amortised and for the step loop alone."""
    from oracle import oracle as ora
    from oracle.cpu_parallel_runner import run_parallel_baseline
    host = os.cpu_count() or 1
    workers = a.cpu_workers or min(host, CPU_WORKER_CAP)
    rate, steps_done, secs, reset_secs = run_parallel_baseline(
        n=a.n, m=a.m, T=a.T, L=a.L, workers=workers, episodes=a.cpu_episodes, epsilon=0.05,
        min_seconds=a.cpu_seconds)
    # second, stronger CPU number: the C oracle env, multi-threaded, random policy (env only)
    c_envs = 4096 if a.n * a.m <= 4096 else 256
    c_secs, _ = ora.rollout_random(c_envs, a.n, a.m, a.T, a.L, 0.5, a.seed, workers, 1)
    return {"value": round(rate, 2), "unit": "env-steps/s", "cores": workers, "kind": "port",
            "host_cores": host, "workers": workers,
            "worker_cap_note": f"batch_size_run = min(os.cpu_count()={host}, {CPU_WORKER_CAP}): the gpurun box "
                               f"allots {CPU_WORKER_CAP} CPUs per GPU while os.cpu_count() reports the whole host",
            "value_step_loop_only": round(steps_done / max(1e-9, secs - reset_secs), 2),
            "value_reset_amortised": round(rate, 2),
            "sample": f"{steps_done // (workers * a.T)} episodes x {workers} subprocess envs x T={a.T} at "
                      f"{a.n}x{a.m} ({steps_done} env-steps, {secs:.1f} s, {reset_secs:.1f} s of it in resets): "
                      f"the reference's ParallelRunner design (Pipe protocol, numpy env, CPU RNN agent + "
                      f"eps-greedy, 1 torch thread; oracle/cpu_parallel_runner.py)",
            "c_env_only": {"value": round(c_envs * a.T / c_secs, 1), "unit": "env-steps/s", "cores": workers,
                           "kind": "port", "sample": f"{c_envs} envs x 1 episode, random policy, C oracle "
                                                     f"(oracle/asg_rollout.c), no agent network"}}


def run_leg(a, dev, world, E, steps, warmup, selector=None, agent=None, count_lsa=False, fused=None, mac="basic_mac",
            use_rnn=None, **extra):
    """Build runner + MAC for one workload and time `steps` transitions after `warmup`.
    Returns elapsed seconds (max over ranks) and mean HIP-event times of the env step, the
    whole selection, and (SAP) the selector kernel alone."""
    from marl_sap_amd import dist as asg_dist
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY

    selector = selector or a.selector
    mac_name = mac
    fused_sched = (a.fused_rollout if fused is None else fused) != 0
    t_setup = time.perf_counter()
    mem0 = leg_memory(dev)
    args = make_args(a, E, selector, agent, fused, mac=mac, use_rnn=use_rnn, **extra)
    runner = r_REGISTRY["gpu"](args, NullLogger())
    env = runner.get_env()
    torch.manual_seed(a.seed)  # identical agent weights on every rank
    mac = mac_REGISTRY[mac](env.scheme, {"agents": a.n}, args)
    mac.to(dev)
    runner.setup(env.scheme, {"agents": a.n}, env.preprocess, mac)

    ev_pairs, sel_pairs, lsa_pairs = [], [], []
    state = {"t": a.T, "timing": False}
    sel_obj = mac.action_selector
    inner = sel_obj.select_action

    import functools

    @functools.wraps(inner)  # keeps the selector's signature: mac.select_actions still passes `out`
    def timed_select(*args_, **kw):  # the selector call alone (SAP: noise + LSA kernel)
        if not state["timing"]:
            return inner(*args_, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = inner(*args_, **kw)
        e1.record()
        lsa_pairs.append((e0, e1, 1))
        return out

    if selector == "sap":
        sel_obj.select_action = timed_select
    elif selector == "bids":  # asg_bids_select alone (the bids transforms, their row store and LSA)
        inner = sel_obj.fused_bids
        sel_obj.fused_bids = timed_select
    fwd_pairs = []
    inner_fwd = env.step_forward

    def timed_forward(*args_, **kw):  # asg_step_forward alone (the step_q schedule's rollout kernel)
        if not state["timing"]:
            return inner_fwd(*args_, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = inner_fwd(*args_, **kw)
        e1.record()
        fwd_pairs.append((e0, e1, 1))
        return out

    env.step_forward = timed_forward

    # the runner's schedule (GpuVecRunner.rollout).  mode "episode" (the default with the fused
    # agent + epsilon-greedy): asg_rollout -- select(0); for t: env.step(t), select(t + 1) -- as one
    # kernel; here it is launched per chunk of steps so that exactly `steps` transitions fall in
    # the timed region (a chunk that stops inside an episode also selects the row after it; the
    # runner itself launches whole episodes).  mode "step": env.step(t) + select(t + 1) fused per
    # step (asg_step_select), the episode's first selection and last step separate.  None:
    # separate env-step and selection launches.  Either way one "step" = one env transition plus
    # one selection (over an episode: T of each).
    fused_pairs = []
    state["selected"] = False

    def timed(pairs, fn, w=1):
        if not state["timing"]:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        pairs.append((e0, e1, w))

    gather_pairs = []

    def new_episode():
        if runner.batch is not None and runner.env.k == a.T:
            # returns gathered on the device; host checks deferred.  Timed with HIP events on the
            # current stream (a collective's work is joined to it before the end event)
            timed(gather_pairs, lambda: runner.finish_episode(sync=False))
        runner.reset(env_reset=False)
        mac.init_hidden(E)
        state["t"] = 0
        state["selected"] = False
        # planned per episode, as GpuVecRunner.rollout does (JumpstartMAC draws its flips here);
        # on the episode schedule the env reset runs in the episode's first launch
        # (asg_reset_rollout), else as its own launch
        with torch.no_grad():
            if selector == "random":
                # the random policy's episode launch (asg_random_rollout), or the split launches
                state["mode"] = "random_episode" if fused_sched else None
            else:
                state["mode"] = mac.fused_mode(env, runner.batch, runner.t_env)
            # (the random policy's launch folds the reset in the Philox mode only: the MT19937 reset
            # is its draw kernels, run by random_rollout itself before the launch); asg_reset_forward
            # for step_q -- asked under no_grad, as the runner's rollout() asks it (the fused
            # paths require inference mode)
            state["fuse_reset"] = bool(a.fuse_reset) and (
                state["mode"] == "episode" or (state["mode"] == "random_episode" and env.rng == "philox")
                or (state["mode"] == "step_q" and mac.fused_reset_ok(env)))
        if not state["fuse_reset"]:
            env.reset(runner.batch, ts=0)

    def advance_random(s_):
        """s_ steps of the random policy (actions + transitions) in one asg_random_rollout launch"""
        t = state["t"]
        rs = t == 0 and state.pop("fuse_reset", False)
        timed(fused_pairs, lambda: env.random_rollout(runner.batch, t, s_, reset=rs), s_)
        if rs and state["timing"]:
            state["fused_resets"] = state.get("fused_resets", 0) + 1
        state["t"] = t + s_

    def advance(s_):
        """s_ transitions (+ their selections) of the current episode in one asg_rollout launch"""
        t = state["t"]
        sf, sl = t == 0, t + s_ < a.T
        with torch.no_grad():
            eps, seed, counter, status, _ = mac.action_selector.fused_params(runner.t_env, False, dev,
                                                                             calls=s_ + sf + sl - 1)

            rs = sf and state.pop("fuse_reset", False)

            def launch():
                mac.hidden_states = env.rollout(runner.batch, t, s_, mac.selector_agent, mac.hidden_states, eps, seed,
                                                counter, status, select_first=sf, select_last=sl, reset=rs)
            timed(fused_pairs, launch, s_)
            if rs and state["timing"]:
                state["fused_resets"] = state.get("fused_resets", 0) + 1
        state["t"] = t + s_

    def one_step():
        t = state["t"]
        with torch.no_grad():
            fused = state["mode"] in ("step", "step_q")
            if selector == "random":
                timed(sel_pairs, lambda: env.random_actions(runner.batch, ts=t))
            elif t == 0 and state.pop("fuse_reset", False):
                # step_q: the reset + the forward on its row (asg_reset_forward), then the selector
                timed(sel_pairs, lambda: mac.fused_reset_select(env, runner.batch, runner.t_env))
            elif not state["selected"]:
                timed(sel_pairs, lambda: runner.select_into_batch(t))
            if fused and t + 1 < a.T:
                timed(fused_pairs, lambda: mac.fused_step_select(env, runner.batch, t, runner.t_env))
                state["selected"] = True
            else:
                timed(ev_pairs, lambda: env.step(runner.batch, ts=t))
                state["selected"] = False
        state["t"] = t + 1

    def run_steps(k):
        while k > 0:
            if state["t"] >= a.T:
                new_episode()
            if state["mode"] in ("episode", "random_episode"):
                s_ = min(k, a.T - state["t"])
                (advance if state["mode"] == "episode" else advance_random)(s_)
                k -= s_
            else:
                one_step()
                k -= 1

    setup_elapsed = time.perf_counter() - t_setup
    tw = time.perf_counter()
    run_steps(warmup)
    asg_dist.barrier()
    torch.cuda.synchronize()
    warm_elapsed = time.perf_counter() - tw
    state["timing"] = True
    t0 = time.perf_counter()
    run_steps(steps)
    torch.cuda.synchronize()
    asg_dist.barrier()
    elapsed = time.perf_counter() - t0
    state["timing"] = False
    if runner.env.k == a.T:
        runner.finish_episode(sync=False)
    runner.flush_pending()  # surfaces any sticky device error of the timed steps
    # mean HIP-event time per step (a launch of w steps counts w)
    mean = lambda prs: sum(p[0].elapsed_time(p[1]) for p in prs) / sum(p[2] for p in prs) if prs else 0.0  # noqa
    res = {"elapsed": elapsed, "warmup_elapsed": warm_elapsed, "kern_ms": mean(ev_pairs), "sel_ms": mean(sel_pairs),
           "lsa_ms": mean(lsa_pairs) if lsa_pairs else None,
           "fused_ms": mean(fused_pairs) if fused_pairs else None, "mode": state.get("mode"),
           "step_forward_ms": mean(fwd_pairs) if fwd_pairs else None,
           "fused_launches": len(fused_pairs), "fused_steps": sum(p[2] for p in fused_pairs),
           "fused_resets": state.get("fused_resets", 0),
           "gather_ms": mean(gather_pairs) if gather_pairs else None, "gathers": len(gather_pairs)}
    if count_lsa and selector in ("sap", "bids") and a.n <= a.m <= 64:
        # one more selection with the step-counting kernel instance.  On the step_q schedule it
        # is a genuine next step (env step t + agent forward + the selection of row t + 1, warm-
        # started from row t's duals, as in the timed window); else a selection on the current row
        with torch.no_grad():
            if state.get("mode") == "step_q":
                if state["t"] + 1 >= a.T:
                    new_episode()
                if state["t"] == 0 and state.pop("fuse_reset", False):
                    mac.fused_reset_select(env, runner.batch, runner.t_env)
                elif not state["selected"]:
                    runner.select_into_batch(state["t"])
                sel_obj.count_steps = torch.zeros(E, dtype=torch.int32, device=dev)
                mac.fused_step_select(env, runner.batch, state["t"], runner.t_env)
            else:
                sel_obj.count_steps = torch.zeros(E, dtype=torch.int32, device=dev)
                t = state["t"] if state["t"] < a.T else 0
                if state["t"] >= a.T:
                    runner.reset()
                    mac.init_hidden(E)
                mac.select_actions(runner.batch, t_ep=t, t_env=runner.t_env)
        # fast-path steps in the low 16 bits, scipy-exact steps (uncertified or rectangular
        # problems) above (asg_sap_select)
        cs = sel_obj.count_steps.long()
        res["path_steps_fast"] = int((cs & 0xFFFF).sum().item())
        res["path_steps_exact"] = int((cs >> 16).sum().item())
        res["exact_problems"] = int(((cs >> 16) > 0).sum().item())
        res["path_steps_per_launch"] = res["path_steps_fast"] + res["path_steps_exact"]
        sel_obj.count_steps = None
    if world > 1:
        # every rank's figures (one all-gather): the job's time is the slowest rank's; the
        # per-rank spread of the kernel time and the per-episode returns all-gather are reported
        # so that a scaling loss can be attributed
        import torch.distributed as tdist
        keys = ("elapsed", "kern_ms", "sel_ms", "fused_ms", "gather_ms")
        mine = torch.tensor([float(res[k] or 0.0) for k in keys], dtype=torch.float64, device=dev)
        if tdist.get_backend() == "gloo":
            mine = mine.cpu()
        allr = torch.empty(world * len(keys), dtype=torch.float64, device=mine.device)
        tdist.all_gather_into_tensor(allr, mine)
        allr = allr.view(world, len(keys)).cpu()
        res["per_rank"] = {k: [round(float(x), 5) for x in allr[:, i]] for i, k in enumerate(keys)}
        res["backend"] = tdist.get_backend()
        res["elapsed"], res["kern_ms"], res["sel_ms"] = (float(allr[:, i].max()) for i in range(3))
    res["global_envs"] = runner.global_envs
    runner.close_env()
    # the timing wrappers are instance attributes closing over bound methods of their own
    # objects (env -> env.step_forward -> env, selector -> select_action -> selector): reference
    # cycles that only the cyclic GC frees.  Break them and collect, so this leg's buffers go
    # back to torch's caching allocator -- and stay there: the next leg's batch (the same 41 GB
    # at configs[2]) reuses the cached block.  No empty_cache(): handing the blocks back to the
    # driver made every leg hipMalloc a fresh 41 GB, and once the never-used VRAM ran out (~7
    # legs) the driver cleared recycled pages on allocation -- a 5.5-6.1 s torch.zeros in a
    # later leg's first episode (round 4's `jumpstart_phase_value` stall)
    env.__dict__.pop("step_forward", None)
    sel_obj.__dict__.pop("select_action", None)
    sel_obj.__dict__.pop("fused_bids", None)
    del runner, mac, env, sel_obj, inner, inner_fwd
    gc.collect()
    torch.cuda.synchronize()
    res["setup_elapsed"] = setup_elapsed
    res["memory"] = {"before": mem0, "after": leg_memory(dev)}
    print(f"[bench] leg envs={E} selector={selector} mac={mac_name} setup {setup_elapsed:.2f} s, warmup "
          f"{warm_elapsed:.3f} s ({warmup} steps), timed {elapsed:.4f} s ({steps} steps), memory {res['memory']}",
          file=sys.stderr, flush=True)
    return res


def real_step_bytes(n, m, L, N, M):
    """Algorithmic HBM bytes of one RealConstellationEnv env-step (per-env
    tables): the L float64 benefit slices read (8nmL) + the int16 actions (2n) read; the float16
    obs rows (2 obs n) and beta (2nmL), bool avail (nm), int16 one-hot (2nm), float16 rewards (2n),
    int16 prev_assigns (2n) written, terminated + filled (9).  The task-major totals and the ranked
    task lists the strip kernel hands the observation kernel are working state, not counted."""
    obs = M * L + N * M * L + (N * M // 2) * L + M
    return 8 * n * m * L + 2 * n + 2 * obs * n + 2 * n * m * L + n * m + 2 * n * m + 2 * n + 2 * n + 9


def real_leg(a, dev, E, steps, warmup, n=324, m=450, T=100, L=3, N=10, M=10):
    """The real-env family's rollout on one GPU: RealConstellationEnv at the
    reference's real_constellation_env.yaml shape (18 x 18 satellites, 450 tasks, T = 100, L = 3,
    N = M = 10), E envs with their own injected benefit tables (sparse, like proximities), random
    policy written into the int16 actions row; `steps` env steps timed after `warmup`, each step =
    the transition + strip + observation kernels (HIP events on the stream)."""
    from marl_sap_amd.components import EpisodeBatch
    from marl_sap_amd.envs import RealAssignEnvBatch
    g = torch.Generator(device=dev).manual_seed(a.seed)
    tables = torch.rand((E, n, m, T), generator=g, device=dev, dtype=torch.float64)
    tables *= torch.rand((E, n, m, 1), generator=g, device=dev, dtype=torch.float64) > 0.8
    env = RealAssignEnvBatch(18, 18, m, T, N, M, L, 0.5, sat_prox_mat=tables, num_envs=E, device=dev)
    del tables
    b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=dev, time_major=True)
    env.reset(b, 0)
    acts = torch.randint(0, m, (warmup + steps, E, n), generator=g, device=dev, dtype=torch.int64).to(torch.int16)
    for t in range(warmup):
        b["actions"][:, t, :, 0] = acts[t]
        env.step(b, t)
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for t in range(warmup, warmup + steps):
        b["actions"][:, t, :, 0] = acts[t]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step(b, t)
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    env.sync()
    step_ms = sum(x.elapsed_time(y) for x, y in ev) / len(ev)
    per = real_step_bytes(n, m, L, N, M) * E
    gbs = per / (step_ms * 1e-3) / 1e9
    pm = pmc_lookup("*pmc_real_step*.json", n=n, m=m, E=E)
    traffic = pm.get("hbm_bytes_per_step") if pm else None
    leg = {"value": round(E * steps / secs, 1), "unit": "env-steps/s", "ms_per_step": round(secs / steps * 1e3, 4),
           "steps": steps, "warmup": warmup, "schedule": "asg_real_step (transition + strip + observation kernels)",
           "workload": f"RealConstellationEnv (real_constellation_env.yaml shape) n={n} satellites, m={m} tasks, T={T}, "
                       f"L={L}, N={N}, M={M}; {E} envs with their own injected float64 tables (80 % of pairs zero), "
                       "random policy, float16 / int16 scheme",
           "envs_per_gpu": E, "kernels_ms": {"real_step": round(step_ms, 4)},
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "traffic_over_algorithmic": round(traffic / per, 4) if traffic else None,
                        "kernel": "asg::real_transition_kernel + real_strip_kernel + real_obs_kernel",
                        "bytes_per_launch": per, "bytes_per_env_step": real_step_bytes(n, m, L, N, M),
                        "pmc_source": os.path.basename(pm["_path"]) if pm else None}}
    if a.cpu_baseline:
        # the C oracle env (oracle/asg_real_oracle.c, one thread) on a bounded sample, as a CPU figure
        import numpy as np
        from oracle import oracle as ora
        rs = np.random.RandomState(0)
        tab = rs.uniform(size=(n, m, T)) * (rs.uniform(size=(n, m, 1)) > 0.8)
        r = ora.OracleRealEnv(tab, N, M, L, 0.5)
        r.reset()
        t1, k = time.perf_counter(), 0
        while time.perf_counter() - t1 < 3.0 and k < T:
            r.step(rs.randint(0, m, size=n))
            k += 1
        leg["cpu_baseline"] = {"value": round(k / (time.perf_counter() - t1), 2), "unit": "env-steps/s", "cores": 1,
                               "kind": "port", "sample": f"{k} steps of one env on the C oracle (3 s bound)"}
    env.close()
    del b, env, acts
    return leg


def leg_memory(dev):
    """Device memory at a leg's edges (GB): torch's allocated / reserved, and free per hipMemGetInfo."""
    free, total = torch.cuda.mem_get_info(dev)
    return {"allocated_gb": round(torch.cuda.memory_allocated(dev) / 1e9, 2),
            "reserved_gb": round(torch.cuda.memory_reserved(dev) / 1e9, 2), "free_gb": round(free / 1e9, 2)}


def res_resets(res):
    """Fused resets per timed step of a leg (asg_reset_rollout launches in the timed window)."""
    return res.get("fused_resets", 0) / res["fused_steps"] if res.get("fused_steps") else 0.0


def sap_kernels(r):
    """HIP-event times per step of a SAP-selector leg: on the step_q schedule the fused env
    step + agent forward (asg_step_forward), the SAP kernel, and the step as a whole (both
    launches plus the selector's host-side work); the episode's first selection (agent kernel
    + SAP) and last env step are separate launches."""
    r4 = lambda v: round(v, 4) if v else None  # noqa: E731
    return {"step_forward": r4(r.get("step_forward_ms")), "sap_select": r4(r.get("lsa_ms")),
            "fused_step_total": r4(r.get("fused_ms")), "env_step": r4(r.get("kern_ms")),
            "first_select": r4(r.get("sel_ms")), "schedule": r.get("mode") or "split"}


def lsa_roofline(a, E, res, kernel="asg::sap_select_kernel", pmc="*pmc_sap_kernel*.json"):
    """SAP selector efficiency: augmenting-path steps (scipy's inner-loop iterations, counted
    by the instrumented kernel instance on one selection) per second of the fused
    noise + LSA kernel, as cycles per step per SIMD.  With a PMC summary of the kernel in
    profiles/ (SQ_INSTS_VALU / SQ_INSTS_SALU per step), against both issue bounds: vector
    (2 cycles per wave64 instruction on a SIMD) and scalar (one scalar unit per CU: 4 cycles
    per instruction per SIMD).  `frac` is the binding issue bound over the measured cycles;
    `bound` names that bound when it explains most of the time (frac >= 0.7), else the
    dependent instruction chain of one step (the serial augmenting path) binds: "latency"."""
    steps, lsa_ms = res.get("path_steps_per_launch"), res.get("lsa_ms")
    if not steps or not lsa_ms:
        return None
    per_s = steps / (lsa_ms * 1e-3)
    cyc = SIMDS * CLOCK_HZ * lsa_ms * 1e-3 / steps
    out = {"bound": None, "kernel": kernel, "kernel_ms": round(lsa_ms, 4),
           "path_steps_per_launch": steps, "path_steps_per_s": round(per_s, 1),
           "path_steps_fast": res.get("path_steps_fast"), "path_steps_exact": res.get("path_steps_exact"),
           "problems_on_exact_solver": res.get("exact_problems"), "problems": E,
           "steps_note": "augmenting-path steps of the certified fast path (column reduction + shortest augmenting "
                         "paths, square problems) and of the scipy-exact solver (uncertified / rectangular problems)",
           "cycles_per_step_per_simd": round(cyc, 1), "achieved": None, "peak": None, "frac": None,
           "unit": "wave-VALU-instr/s", "traffic": None}
    pm = pmc_lookup(pmc, n=a.n, m=a.m, E=E)
    if pm and pm.get("valu_insts_per_path_step"):
        vps = pm["valu_insts_per_path_step"]
        sps = pm.get("salu_insts_per_path_step") or 0.0
        peak = SIMDS * CLOCK_HZ / VALU_CYCLES_PER_WAVE_INSTR
        ach = vps * per_s
        vb, sb = vps * VALU_CYCLES_PER_WAVE_INSTR, sps * 4
        bind = max(vb, sb)
        frac = bind / cyc
        out.update({"achieved": round(ach / 1e9, 2), "peak": round(peak / 1e9, 2), "unit": "G wave-VALU-instr/s",
                    "valu_frac": round(ach / peak, 4), "valu_insts_per_path_step": round(vps, 2),
                    "valu_bound_cycles_per_step": round(vb, 1),
                    "salu_insts_per_path_step": round(sps, 2), "salu_bound_cycles_per_step": round(sb, 1),
                    "salu_frac": round(sb / cyc, 4), "frac": round(frac, 4),
                    "bound": ("salu-issue" if sb >= vb else "valu-issue") if frac >= 0.7 else "latency",
                    "pmc": os.path.basename(pm.get("_path", "")) or None})
        for k in ("wait_any_frac", "wait_inst_any_frac", "active_inst_any_frac", "resident_waves_per_simd"):
            if k in pm:
                out[k] = round(pm[k], 3)
    return out


def main():
    a = parse()
    from marl_sap_amd import dist as asg_dist
    rank, world = asg_dist.init_from_env()
    # CPU baseline first: its worker processes are forked before this process touches the GPU
    cpu = cpu_baseline(a) if rank == 0 and world == 1 and a.cpu_baseline else None

    local = asg_dist.local_device_index()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    E = a.envs
    res = run_leg(a, dev, world, E, a.steps, a.warmup, count_lsa=True)
    G = res["global_envs"]
    value = G * a.steps / res["elapsed"]
    kern_ms, sel_ms = res["kern_ms"], res["sel_ms"]
    if res.get("mode") == "step_q" and res.get("step_forward_ms"):
        bids = a.selector == "bids"
        roof = fused_roofline(a, E, res["step_forward_ms"], use_rnn=a.use_rnn and not bids, q_out=True, bids=bids)
    elif res.get("mode") == "random_episode" and res.get("fused_ms"):
        roof = random_roofline(a, E, res["fused_ms"], res_resets(res))
    elif res.get("fused_ms"):
        roof = fused_roofline(a, E, res["fused_ms"], resets_per_step=res_resets(res))
    else:
        per_launch = step_bytes(a.n, a.m, a.L) * E
        achieved = per_launch / (kern_ms * 1e-3) / 1e9
        pm = pmc_lookup("*pmc_step_kernel*.json", n=a.n, m=a.m, E=E, L=a.L)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pm.get("hbm_bytes_per_launch") if pm else None,
                "kernel": "asg::step_kernel", "kernel_ms": round(kern_ms, 4), "bytes_per_launch": per_launch}

    secondary = a.secondary if a.secondary >= 0 else int(world == 1 and a.config in (2, 3))
    extra = {}

    def leg_base(r, sk, sw):
        return {"value": round(r["global_envs"] * sk / r["elapsed"], 1), "unit": "env-steps/s",
                "ms_per_step": round(r["elapsed"] / sk * 1e3, 4), "steps": sk, "warmup": sw,
                "schedule": r.get("mode") or "split"}

    if secondary:
        # at least one episode per leg, so the window holds a reset at the rate of the profiled
        # whole-episode launches (fused_roofline's traffic accounting)
        sk, sw = max(a.T, a.steps // 2), max(5, a.warmup // 2)
        if a.selector != "random":
            r2 = run_leg(a, dev, world, E, sk, sw, selector="eps", agent="rnn_torch")
            extra["pytorch_agent"] = {
                **leg_base(r2, sk, sw),
                "what": "agent rnn_torch (the explicit opt-out): BasicMAC + the plain PyTorch RNNAgent module "
                        "(hipBLASLt linears + GRUCell, fp32) + asg_epsilon_greedy kernel, same env step",
                "select_ms": round(r2["sel_ms"], 4), "env_step_ms": round(r2["kern_ms"], 4)}
        if a.selector == "eps" and a.agent in FUSED_AGENTS:
            # the other schedules of the same workload: one fused launch per step, and separate
            # env-step + agent launches
            r4 = run_leg(a, dev, world, E, sk, sw, fused=3)
            extra["step_rollout"] = {
                **leg_base(r4, sk, sw), "fused_step_select_ms": round(r4["fused_ms"], 4) if r4["fused_ms"] else None,
                "env_step_ms": round(r4["kern_ms"], 4) if r4["kern_ms"] else None,
                "select_ms": round(r4["sel_ms"], 4) if r4["sel_ms"] else None,
                "what": "same workload, asg_rollout launched per step (env step t + agent forward + eps-greedy for "
                        "t + 1) for T - 1 of T steps, the episode's first selection and last step separate"}
            r6 = run_leg(a, dev, world, E, sk, sw, fused=0)
            extra["split_rollout"] = {
                **leg_base(r6, sk, sw), "env_step_ms": round(r6["kern_ms"], 4), "select_ms": round(r6["sel_ms"], 4),
                "what": "same workload with --fused-rollout 0: asg_step then the fused agent forward + eps-greedy "
                        "kernel (rnn_agent_h2_kernel), one launch each per step"}
        if a.n <= a.m <= 64 and a.selector != "sap":
            r3 = run_leg(a, dev, world, E, sk, sw, selector="sap", agent="rnn", count_lsa=True)
            extra["sap"] = {
                **leg_base(r3, sk, sw),
                "what": "SequentialAssignmentProblemSelector (eps 0.05) on the step_q schedule: per step one "
                        "asg_step_forward launch (env step t + the RNNAgent forward of t + 1, Q to HBM) and one "
                        "asg_sap_select_into launch (per-env Gaussian noise + scipy-exact LSA, one wave64 per env, "
                        "actions written into the batch row)",
                "kernels_ms": sap_kernels(r3),
                "roofline_lsa": lsa_roofline(a, E, r3)}
            if r3.get("mode") == "step_q" and r3.get("step_forward_ms"):
                extra["sap"]["roofline_step_forward"] = fused_roofline(a, E, r3["step_forward_ms"],
                                                                       use_rnn=a.use_rnn, q_out=True)
        if a.config == 2 and world == 1 and a.selector == "eps":
            # config/algs/ippo_sap.yaml's env path: bids_as_actions + the continuous selector over
            # softmaxed pi_logits (Linear agent): per step asg_step_forward (env step t with the
            # assignments of the bids row t + the agent forward of t + 1, Q written) and
            # asg_bids_select (pi_logits softmax, softmax over the agents, noise, the bids row, its LSA);
            # the same with separate launches beside it
            for name, fz in (("ippo_sap", None), ("ippo_sap_split", 0)):
                rb = run_leg(a, dev, world, E, sk, sw, selector="bids", agent="rnn", fused=fz, count_lsa=fz is None)
                extra[name] = {
                    **leg_base(rb, sk, sw),
                    "what": "ippo_sap.yaml env path: bids_as_actions, ContinuousActionSelector (softmax_agent_inputs, "
                            "std 0.3 -> 0.05 over 50,000 env steps) on pi_logits of the Linear RNNAgent; "
                            + ("step_q schedule: asg_step_forward + asg_bids_select per step" if fz is None else
                               "separate launches: the agent kernel, asg_bids_select, asg_step per step"),
                    "kernels_ms": {"step_forward": round(rb["step_forward_ms"], 4) if rb.get("step_forward_ms") else None,
                                   "bids_select": round(rb["lsa_ms"], 4) if rb.get("lsa_ms") else None,
                                   "fused_step_total": round(rb["fused_ms"], 4) if rb.get("fused_ms") else None,
                                   "env_step": round(rb["kern_ms"], 4) if rb["kern_ms"] else None,
                                   "select": round(rb["sel_ms"], 4) if rb["sel_ms"] else None}}
                if rb.get("mode") == "step_q" and rb.get("step_forward_ms"):
                    extra[name]["roofline_step_forward"] = fused_roofline(a, E, rb["step_forward_ms"], use_rnn=False,
                                                                          q_out=True, bids=True)
                if fz is None:
                    # bids_select_kernel: the two softmaxes (2n wave reductions), the noise, the bids row
                    # store, then the LSA of the negated bids -- augmenting-path steps counted by its
                    # instrumented instance on one more step of the same schedule
                    extra[name]["roofline_lsa"] = lsa_roofline(a, E, rb, kernel="asg::bids_select_kernel",
                                                               pmc="*pmc_bids_kernel*.json")
            # the reference's own algorithms for this env (config/algs/mock_constellation_*.yaml):
            # jumpstart_mac with the HAA jumpstart selector, use_rnn: False (Linear + ReLU agent),
            # jumpstart epsilon 1 -> 0 over 20,000 env steps -- one 16,384-env episode is 327,680
            # env steps, so the warmup episode is the jumpstart (HAA) phase and the timed steps run
            # the RL selector
            js = dict(mac="jumpstart_mac", use_rnn=False, jumpstart_action_selector="haa_selector",
                      jumpstart_epsilon_start=1.0, jumpstart_epsilon_finish=0.0, jumpstart_epsilon_anneal_time=20000,
                      jumpstart_evaluation_epsilon=0.0)
            for name, sel_, yaml in (("iql", "eps", "mock_constellation_iql.yaml"),
                                     ("reda", "sap", "mock_constellation_reda.yaml")):
                eps_over = dict(epsilon_start=1.0, epsilon_finish=0.0, epsilon_anneal_time=20000)
                # two warmup episodes: the jumpstart (HAA) one at t_env = 0, then one RL episode, so the
                # timed episodes are the steady state (the RL path's first-use allocations -- the Q
                # buffer, the warm-start duals -- happen in the warmup, as in any longer run)
                rj = run_leg(a, dev, world, E, sk, 2 * a.T, selector=sel_, agent="rnn", count_lsa=sel_ == "sap", **js,
                             **eps_over)
                extra[name] = {
                    **leg_base(rj, sk, a.T),
                    "what": f"{yaml}: jumpstart_mac (haa_selector jumpstart) + "
                            f"{'epsilon_greedy' if sel_ == 'eps' else 'sap'} selector, RNNAgent use_rnn False "
                            f"(Linear + ReLU, fused split-f16 kernel), both epsilons 1 -> 0 over 20,000 env steps; "
                            f"timed after two warmup episodes (the jumpstart/HAA phase at t_env = 0, then one RL "
                            f"episode)",
                    "warmup_value": round(rj["global_envs"] * 2 * a.T / rj["warmup_elapsed"], 1),
                    "kernels_ms": sap_kernels(rj) if sel_ == "sap" else {
                        "fused_rollout_per_step": round(rj["fused_ms"], 4) if rj["fused_ms"] else None,
                        "env_step": round(rj["kern_ms"], 4) if rj["kern_ms"] else None,
                        "select": round(rj["sel_ms"], 4) if rj["sel_ms"] else None}}
                if sel_ == "sap":
                    extra[name]["roofline_lsa"] = lsa_roofline(a, E, rj)
                if rj.get("mode") == "step_q" and rj.get("step_forward_ms"):
                    extra[name]["roofline"] = fused_roofline(a, E, rj["step_forward_ms"], use_rnn=False, q_out=True)
                elif rj.get("fused_ms"):
                    extra[name]["roofline"] = fused_roofline(a, E, rj["fused_ms"], use_rnn=False,
                                                             resets_per_step=res_resets(rj))
        if a.config == 2 and world == 1:
            # BASELINE configs[4] on this GPU: 256 x 256 dense benefits, 2,048 envs, the same
            # BasicMAC + RNNAgent + eps-greedy on the fused rollout schedule
            c4 = argparse.Namespace(**vars(a))
            for k in ("n", "m", "envs", "benefits"):
                setattr(c4, k, CONFIGS[4][k])
            c4.config = 4
            r5 = run_leg(c4, dev, world, c4.envs, sk, sw)
            leg = {**leg_base(r5, sk, sw),
                   "workload": CONFIGS[4]["label"] + f"; T={a.T}, L={a.L}, BasicMAC+rnn(GRU 64, fp32, fused kernel) + "
                                                     "epsilon-greedy 0.05, dense benefits",
                   "envs_per_gpu": c4.envs, "n": c4.n, "m": c4.m,
                   "kernels_ms": {"fused_rollout_per_step": round(r5["fused_ms"], 4) if r5.get("fused_ms") else None,
                                  "env_step": round(r5["kern_ms"], 4) if r5["kern_ms"] else None,
                                  "select": round(r5["sel_ms"], 4) if r5["sel_ms"] else None}}
            if r5.get("fused_ms"):
                leg["roofline"] = fused_roofline(c4, c4.envs, r5["fused_ms"], resets_per_step=res_resets(r5))
            extra["config4"] = leg
            # BASELINE configs[1]: 16 x 16, 4,096 envs, random policy (asg_random_actions + asg_step
            # per step; SURVEY §8(d) B_env = 6,729 B per env-step, B_step with the fused one-hot 7,753)
            c1 = argparse.Namespace(**vars(a))
            for k in ("n", "m", "envs", "benefits", "selector"):
                setattr(c1, k, CONFIGS[1][k])
            c1.config = 1
            # the random policy's episode launch (asg_random_rollout: reset + T x (actions +
            # transition) in one launch), with the split launches (asg_random_actions + asg_step per
            # step) beside it
            r1 = run_leg(c1, dev, world, c1.envs, max(sk, 4 * a.T), sw)
            sk1 = max(sk, 4 * a.T)
            extra["config1"] = {
                **leg_base(r1, sk1, sw),
                "workload": CONFIGS[1]["label"] + f"; T={a.T}, L={a.L}: asg_random_rollout (the episode's reset, "
                                                  "uniform actions and transitions in one launch)",
                "envs_per_gpu": c1.envs, "n": c1.n, "m": c1.m,
                "kernels_ms": {"random_rollout_per_step": round(r1["fused_ms"], 4) if r1.get("fused_ms") else None},
                "roofline": random_roofline(c1, c1.envs, r1["fused_ms"], res_resets(r1)) if r1.get("fused_ms") else None}
            r1s = run_leg(c1, dev, world, c1.envs, sk, sw, fused=0)
            sb = step_bytes(c1.n, c1.m, c1.L) * c1.envs
            gbs = sb / (r1s["kern_ms"] * 1e-3) / 1e9 if r1s["kern_ms"] else None
            extra["config1_split"] = {
                **leg_base(r1s, sk, sw),
                "workload": CONFIGS[1]["label"] + f"; T={a.T}, L={a.L}: asg_random_actions + asg_step per step",
                "kernels_ms": {"env_step": round(r1s["kern_ms"], 4) if r1s["kern_ms"] else None,
                               "random_actions": round(r1s["sel_ms"], 4) if r1s["sel_ms"] else None},
                "env_step_roofline": {"kernel": "asg::step_kernel", "unit": "GB/s",
                                      "achieved": round(gbs, 1) if gbs else None,
                                      "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None, "bytes_per_launch": sb,
                                      "note": "one launch per step: 4,096 envs x 7.75 KB = 32 MB per launch, "
                                              "launch-bound"}}
            # the same-seed mode (rng="mt19937": env e replays numpy's legacy stream seeded with
            # seed + e, the reference's draws) on the episode kernel: configs[2] with the handle's
            # float32 benefit table read for the lookahead rows (the float64 rewards evaluated from
            # the reset's recorded MT19937 draws, which the reset writes with that table)
            rc = run_leg(a, dev, world, E, sk, sw, env_rng="mt19937")
            leg = {**leg_base(rc, sk, sw),
                   "workload": "configs[2] in the same-seed mode: rng mt19937 (per env np.random.seed(seed + env)), "
                               "float32 benefit table + recorded draws; asg_reset (MT19937 draws, table write) + the "
                               "episode kernel",
                   "kernels_ms": {"fused_rollout_per_step": round(rc["fused_ms"], 4) if rc.get("fused_ms") else None,
                                  "fused_note": "the episode launches of the window, their asg_reset (table draws) "
                                                "included"}}
            if rc.get("fused_ms"):
                tb = 4 * a.n * a.m * E  # one float32 table slice read per env-step (+ its write at the reset)
                pb = 32 * a.n * a.m * E // a.T  # the draws (16 B per pair) written and read once per episode
                croof = fused_roofline(a, E, rc["fused_ms"], resets_per_step=res_resets(rc))
                per = croof["bytes_per_launch"] + 2 * tb + pb
                croof.update({"bytes_per_launch": per, "achieved": round(per / (rc["fused_ms"] * 1e-3) / 1e9, 1),
                             "frac": round(per / (rc["fused_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "traffic": None, "kernel": "asg::rollout_kernel<TAB> (+ asg_reset's table draws)",
                             "per_launch_note": "the Philox accounting + 4nm per env-step of table read (one new "
                                                "float32 slice per step) + 4nm of table write (the reset's T slices "
                                                "over T steps) + 32nm / T of draws (written and read once per "
                                                "episode)"})
                croof.pop("traffic_pmc", None)
                croof.pop("traffic_over_algorithmic", None)
                croof.pop("traffic_note", None)
                croof.pop("issue", None)
                croof.pop("survey_b_batch", None)
                # PMC bytes of the same launches (tools/gpu_r6.sh compat_pmc: separate FETCH / WRITE
                # passes over one whole same-seed episode: the draw kernel, the table kernel, the episode
                # kernel with its reset row), per step with this window's reset share
                pm = pmc_lookup("*pmc_rollout_tab*.json", n=a.n, m=a.m, E=E, L=a.L)
                if pm:
                    ks = pm.get("kernels", {})
                    col = "hbm_bytes_fetch_doubled"
                    roll = next((v[col] for k, v in ks.items() if "rollout_kernel" in k), None)
                    draw = sum(v[col] for k, v in ks.items() if "mt_reset_kernel" in k or "mt_table_kernel" in k)
                    if roll:
                        spl = pm.get("steps_per_launch", a.T)
                        rb = reset_bytes(a.n, a.m, a.L) * E
                        rps = res_resets(rc)
                        tr = round((roll - rb) / spl + rps * (rb + draw))
                        table_read = next((v for k, v in pm.get("table_reads", {}).items()), None)
                        croof.update({"traffic": tr, "traffic_over_algorithmic": round(tr / per, 4),
                                      "traffic_pmc": os.path.basename(pm["_path"]),
                                      "traffic_note": "(2 FETCH_SIZE + WRITE_SIZE) of the episode kernel per step, its "
                                                      "reset row replaced by this window's share, + the draw and table "
                                                      "kernels' bytes per reset amortised the same way",
                                      "episode_kernel_bytes_per_step": round((roll - rb) / spl)})
                        if table_read:
                            croof["table_read_over_algorithmic"] = table_read
                leg["roofline"] = croof
            extra["compat"] = leg
        if a.config == 2 and world == 1:
            # SURVEY §8(f) rows 1 and 3 on this GPU (tools/bench_aux.py): the SAP learner's B x (T-1)
            # target LSAs as one asg_lsa_batched launch (the reference: a serial scipy loop,
            # sap_q_learner.py:98-108, timed beside it on the host), and the device ReplayBuffer's
            # insert of a 4,096-episode rollout batch + a 32-episode sample (episode_buffer.py:237-277)
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import bench_aux
            lt = bench_aux.bench_sap_targets(32, a.T + 1, a.n, a.m, dev)
            extra["learner_lsa_targets"] = {
                **lt, "what": "sap_q_learner.py:98-108's per-(episode, t) scipy LSA on the target Q-values: "
                              "marl_sap_amd.learners.sap_target_max_qvals (one asg_lsa_batched launch + gather), "
                              "32 episodes x (T-1) problems of n x m; scipy_loop_ms = the reference's loop on the host"}
            rp = bench_aux.bench_replay(4096, 8192, a.n, a.m, a.T, a.L, 32, dev)
            rp["insert_frac"] = round(rp["insert_GBps"] / HBM_PEAK_GBS, 4)
            rp["what"] = ("device ReplayBuffer (episode_buffer.py:237-277 layout): insert_episode_batch of one "
                          "4,096-env time-major rollout batch into an 8,192-episode ring (bytes read + written), "
                          "sample(32)")
            extra["replay_buffer"] = rp
        if a.config == 2 and world == 1 and a.real_envs > 0:
            # the real-env family at its reference shape; last, with the
            # allocator's cache released first (its per-env tables and 101-row batch are the largest
            # allocation of the run)
            gc.collect()
            torch.cuda.empty_cache()
            extra["real"] = real_leg(a, dev, a.real_envs, 20, 5)

    if a.selector == "random":
        ra = None
    elif res.get("fused_ms"):
        # the separate agent kernel only runs the episode's first selection here (h = 0, the
        # W_hh products skipped): its figure comes from the split-schedule leg when it ran
        sp = extra.get("split_rollout")
        ra = agent_roofline(a, E, sp["select_ms"], "asg::rnn_agent_h2_kernel (forward + eps-greedy), "
                            "split-schedule leg") if sp and sp.get("select_ms") else None
    elif a.selector == "sap":
        ra = agent_roofline(a, E, sel_ms - (res["lsa_ms"] or 0.0), f"{a.agent} forward")
    else:
        ra = agent_roofline(a, E, sel_ms, "asg::rnn_agent_h2_kernel (forward + eps-greedy)"
                            if a.agent in FUSED_AGENTS else "torch RNNAgent + asg_epsilon_greedy")
    if rank == 0:
        sel_name = {"eps": "epsilon-greedy", "sap": "SAP", "random": "random",
                    "bids": "continuous (bids_as_actions, ippo_sap.yaml)"}[a.selector]
        line = {
            "metric": f"env steps/sec (whole node), {a.n}-agent assignment env, 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(res["elapsed"] / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic (Philox {a.benefits} benefits, random-init RNN agent)",
            "config": {"workload": CONFIGS[a.config]["label"] + f"; T={a.T}, L={a.L}, BasicMAC+{a.agent}"
                                   f"({'GRU' if a.use_rnn else 'Linear'} 64, fp32) + {sel_name} selector, "
                                   f"{a.benefits} benefits",
                       "baseline_config_index": 3 if (a.config == 2 and world > 1) else a.config,
                       "envs_per_gpu": E, "global_envs": G, "n": a.n, "m": a.m, "T": a.T, "L": a.L,
                       "parallelism": f"env-sharded x{world} (gather of returns per episode)"},
            "roofline": roof,
            "kernels_ms": {**(sap_kernels(res) if a.selector == "sap" else {
                               "step_forward": round(res["step_forward_ms"], 4) if res.get("step_forward_ms") else None,
                               "bids_select": round(res["lsa_ms"], 4) if res.get("lsa_ms") else None,
                               "fused_step_total": round(res["fused_ms"], 4) if res.get("fused_ms") else None,
                               "env_step": round(kern_ms, 4) if kern_ms else None,
                               "select": round(sel_ms, 4) if sel_ms else None} if a.selector == "bids" else {
                               "fused_rollout_per_step": round(res["fused_ms"], 4) if res.get("fused_ms") else None,
                               "env_step": round(kern_ms, 4) if kern_ms else None,
                               "select": round(sel_ms, 4) if sel_ms else None}),
                           "schedule": res.get("mode") or "split",
                           "fused_launches": res.get("fused_launches"), "fused_steps": res.get("fused_steps"),
                           "note": {"episode": "asg_rollout: each launch runs a chunk of an episode's steps (the "
                                               "runner launches whole episodes); kernel time per step",
                                    "step": "T-1 fused launches + 1 select + 1 step per episode",
                                    "step_q": "per episode: T-1 x (asg_step_forward + asg_sap_select_into), "
                                              "1 select (agent kernel + SAP) + 1 step"}.get(
                                        res.get("mode"), "one select + one step per step")},
            "roofline_agent": ra,
            "cpu_baseline": cpu,
        }
        if world > 1:
            pr = res["per_rank"]
            kern = pr["fused_ms"] if any(pr["fused_ms"]) else pr["kern_ms"]
            line["multi_rank"] = {
                "backend": res["backend"],
                "backend_note": "torch.distributed backend initialised ('nccl' is RCCL on ROCm)",
                "kernel": "fused_rollout_per_step" if any(pr["fused_ms"]) else "env_step",
                "kernel_ms_max": max(kern), "kernel_ms_min": min(kern),
                "all_gather_returns_ms_max": max(pr["gather_ms"]), "all_gather_returns_ms_min": min(pr["gather_ms"]),
                "gathers_per_rank": res.get("gathers"),
                "elapsed_s_per_rank": pr["elapsed"], "kernel_ms_per_rank": kern,
                "all_gather_returns_ms_per_rank": pr["gather_ms"],
                "note": "HIP-event times per rank: the kernel per step, and GpuVecRunner.finish_episode (the "
                        "per-episode all-gather of the float64 returns) per episode inside the timed window"}
        if a.selector == "sap":
            line["roofline_lsa"] = lsa_roofline(a, E, res)
        elif a.selector == "bids":
            line["roofline_lsa"] = lsa_roofline(a, E, res, kernel="asg::bids_select_kernel", pmc="*pmc_bids_kernel*.json")
        if extra:
            line["secondary"] = extra
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
