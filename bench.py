#!/usr/bin/env python3
"""bench.py -- self-play moves/sec at 200 sims/move on a 15x15 board (BASELINE.json).

Workload (BASELINE config 2, per GPU): 4096 concurrent self-play games from the
empty board, 200 simulations per move, medium difficulty (c_puct 1.6,
exploration 0.05), beta = 0, planner_steps = 0, random-init network weights
(numpy default_rng(0)), continuous refill of finished games.

Measured in steady state: every slot first plays --burn-in plies (default 600)
without the PV forward -- the moves are the same, the search never reads the
priors -- so the timed window sees continuous refill's mix of game plies (opening
plies included) rather than the synchronised start of 4096 fresh games (the two
halves of the timed window agree within 0.3 %).

One "step" = every game slot plays `--plies-per-step` plies (one kernel launch,
one wavefront per game) followed by the policy-value forward of EVERY node
those searches created -- the GomokuModel.predict calls the reference makes
(ai_agent.py:522-523) -- logits, value, softmax and the masked prior
(ai_agent.py:564-582), and (N > 1) the sync-free all-gather of the finished
games' (s, pi, z) records (gzero.dist.RecordExchange, RCCL).  `value` counts
every ply played by every rank.

The PV forward (default --pv-mode tree) is gz_pv_forward_tree: each search
root runs the full f16x3 tower (3-term fp16 split on MFMA, f32 accumulate) and
keeps its maps and pre-BN accumulators (bit-identical to --pv-mode full); each
root child is the root's accumulators plus the convolution of its one-stone input
differences (pv_dg_kernel) and each grandchild recomputes the windows its stone
changes from its parent's squares (pv_sib_kernel): within 2e-5 of the full
forward's logits / value (1e-4 of the reference's fp32 forward).
--pv-precision fp32 runs the exact-f32 MFMA kernel.

Also reported: the roofline of the PV forward (executed MFMA FLOP / kernel time,
and the full-forward-equivalent rate), config 4 (planner plies) and the exact-fp32
run as labelled secondaries, the prior-elided MCTS-only rate (moves identical
without the priors), and the CPU baseline: the C oracle + torch-fp32 forwards
("port") on the host cores -- P processes x 1 thread, 1 process x P threads, and
config 1.
Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1 either under torchrun
(one rank per GPU from its env) or self-launched: without WORLD_SIZE in the
environment, bench.py starts `python -m torch.distributed.run --nproc-per-node N`
as a child process and relays rank 0's line.  The line's `distributed` block names
the backend, the world size and every rank's device (PCI address).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "alphazero-gomoku_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gzero import _lib  # noqa: E402
from gzero import dist as gdist  # noqa: E402
from gzero import weights  # noqa: E402
from gzero.device import PVWeights, ptr, stream  # noqa: E402
from gzero.selfplay import COUNTER_DTYPE, SelfPlayEngine  # noqa: E402

METRIC = "self-play moves/sec at 200 sims/move, 15x15 board, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 / 32x32x2 dense peak
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense fp16/bf16 MFMA peak (spec)
PV_FLOP = 2 * weights.PV_MACS  # 267.38 MFLOP per board
TILETAP_FLOP = 2 * 16 * 128 * 128  # one 16-row tile x one tap of a residual 3x3 conv (fp32-equivalent)
# per incremental node besides its residual tiles: conv0 (one 16-row tile, K 27), the
# 1x1 head convs on the radius-5 square (121 rows unclipped) and the FC heads
INC_EXTRA_FLOP = 2 * (16 * 128 * 27 + 121 * 128 * 3 + 450 * 225 + 225 * 64 + 64)



def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_traffic(boards, mode):
    """HBM bytes per PV launch of `boards` boards: rocprof 2 x FETCH_SIZE + WRITE_SIZE per
    board of the same PV mode (profiles/pv_traffic.json, profiles/collect.sh) x boards, or None."""
    p = os.path.join(REPO, "profiles", "pv_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        if d.get("bytes_per_board") and d.get("pv_mode", "full") == mode:
            return round(d["bytes_per_board"] * boards, 1), d
    return None, None


def load_clock(kernel):
    """Measured shader clock and MFMA-busy share of `kernel` under load (newest
    profiles/rNN/clock.json that has it), or None."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        p = os.path.join(REPO, "profiles", rnd, "clock.json")
        if os.path.exists(p):
            with open(p) as f:
                k = json.load(f).get("kernels", {}).get(kernel)
            if k:
                return dict(k, source=f"profiles/{rnd}/clock.json (rocprofv3 GRBM_GUI_ACTIVE / duration)")
    return None


def _cpu_worker(task):
    """One host process of the CPU baseline: the C oracle's search (1 thread) of
    MCTS plies from a start position, then the torch-fp32 CPU forwards (`threads`
    intra-op threads) of every node those searches created -- the reference's
    per-ply work (ai_agent.py:168-204 + GomokuModel.predict per node).  With
    planner_steps > 0 every rollout starts with BG-planner plies whose GraphNet +
    OpponentDQN forwards also run on torch CPU (bg_planner.py:243-250)."""
    positions, sims, seed, budget, threads, beta, planner_steps = task
    import torch as T
    T.set_num_threads(threads)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from gzero.boards import words_to_cells, planes_from_cells

    def start(k):  # the k-th start position (cycled); a finished game moves to the next
        black, white, n_moves, player, gid = positions[k % len(positions)]
        cells = words_to_cells(black, white)
        b = O.Board()
        O.lib().or_board_init(b)
        for i in range(225):
            b.cell[i] = int(cells[i])
        b.n_moves, b.player = int(n_moves), int(player)
        return b, gid

    k = 0
    b, gid = start(k)
    net = weights.PolicyValueNet()
    net.load_state_dict(weights.init_state_dict(0))
    net.eval()
    pq = None
    if planner_steps:
        from gzero import planner_nets
        gn, dq = planner_nets.GraphNet(), planner_nets.OpponentDQN()
        gn.load_state_dict(planner_nets.init_graphnet_state(0))
        dq.load_state_dict(planner_nets.init_dqn_state(1))
        gn.eval()
        dq.eval()

        def pq(board, game_id, sim, step):
            x = T.from_numpy(planes_from_cells(np.frombuffer(bytes(board.cell), dtype=np.int8)[None]))
            with T.no_grad():
                return T.softmax(gn(x), dim=1)[0].numpy(), dq(x)[0].numpy()
    p = O.make_params("medium", sims=sims, beta=beta, seed=seed, planner_steps=planner_steps, pq=pq)
    t0 = time.perf_counter()
    plies = predicts = 0
    while time.perf_counter() - t0 < budget:
        if b.over:
            k += 1
            b, gid = start(k)
        root = np.frombuffer(bytes(b.cell), dtype=np.int8).copy()
        mv, tree = O.get_move(b, b.player, p, gid, cap=4096)
        # the forwards of this ply's nodes: every node's board (root + path stones);
        # terminal nodes are not forwarded (predicts counts the non-terminal ones)
        par, mvs = tree["parent"], tree["move"]
        if not par:  # an opening ply (_opening_move, ai_agent.py:138-166): no search, no forwards
            plies += 1
            O.lib().or_make_move(b, mv // 15, mv % 15)
            continue
        nb = np.zeros((len(par), 225), np.int8)
        col = np.zeros(len(par), np.int8)
        nb[0], col[0] = root, 3 - b.player
        for i in range(1, len(par)):
            nb[i] = nb[par[i]]
            col[i] = 3 - col[par[i]]
            nb[i, mvs[i]] = col[i]
        n = min(tree["predicts"], len(par))
        x = T.from_numpy(planes_from_cells(nb[:n]))
        with T.no_grad():
            for i in range(0, n, 64):
                net(x[i:i + 64])
        predicts += n
        plies += 1
        O.lib().or_make_move(b, mv // 15, mv % 15)
    return plies, predicts, time.perf_counter() - t0


def _cpu_warm(_):
    """Pool start-up: import torch and the oracle in each worker before any timing."""
    import torch as T
    T.set_num_threads(1)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: F401
    return 0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """(CPUs this process may run on, the CPU share the worker pool is sized to).  On
    the GPU box the affinity mask shows the whole machine; the job's share is the
    OMP_NUM_THREADS the box sets (16 per GPU)."""
    aff = len(os.sched_getaffinity(0))
    share = aff
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) < aff:
        share = int(env)
    return aff, share


def cpu_baseline(pool, procs, positions, sims, seed, budget_s):
    """The reference's CPU self-play work on the GPU box's host cores,
    three bounded runs:
      1. config 2 work, `procs` processes x 1 thread, each from one of the GPU run's
         timed-window start positions (the headline value: the best aggregate);
      2. config 2 work, 1 process x `procs` torch threads;
      3. config 1 (1 game from the empty board, 50 sims, beta 0.2, planner_steps 5,
         medium), 1 process x `procs` torch threads.
    value = plies / wall time of each run."""
    aff, _ = host_cores()
    cpu = cpu_model()
    runs = []
    # worker i starts at position i and moves on through the list when its game ends
    tasks = [(positions[i:] + positions[:i], sims, seed, budget_s, 1, 0.0, 0) for i in range(procs)]
    t0 = time.perf_counter()
    res = pool.map(_cpu_worker, tasks)
    wall = time.perf_counter() - t0
    plies, predicts = sum(r[0] for r in res), sum(r[1] for r in res)
    runs.append({"run": f"config 2 work: {procs} processes x 1 thread", "value": plies / wall, "unit": "moves/s",
                 "per_core": plies / wall / procs, "plies": plies, "forwards": predicts, "wall_s": round(wall, 2),
                 "cores": procs})
    one = pool.apply(_cpu_worker, ((positions, sims, seed, budget_s, procs, 0.0, 0),))
    runs.append({"run": f"config 2 work: 1 process x {procs} threads", "value": one[0] / one[2], "unit": "moves/s",
                 "per_core": one[0] / one[2] / procs, "plies": one[0], "forwards": one[1],
                 "wall_s": round(one[2], 2), "cores": procs})
    empty = [(np.zeros(8, np.uint32), np.zeros(8, np.uint32), 0, 1, g) for g in range(4)]
    c1 = pool.apply(_cpu_worker, ((empty, 50, seed, budget_s, procs, 0.2, 5),))
    runs.append({"run": f"config 1 (50 sims, beta 0.2, planner_steps 5, medium) from the empty board; 1 process x {procs} threads",
                 "value": c1[0] / c1[2], "unit": "moves/s", "per_core": c1[0] / c1[2] / procs, "plies": c1[0],
                 "forwards": c1[1], "wall_s": round(c1[2], 2), "cores": procs})
    for r in runs:
        r["value"] = round(r["value"], 3)
        r["per_core"] = round(r["per_core"], 4)
    return {
        "value": runs[0]["value"],
        "unit": "moves/s",
        "cores": int(procs),
        "kind": "port",
        "cpu": cpu,
        "host_cpus_in_affinity": aff,
        "sample": (f"run 1 of `runs`: {procs} processes x 1 thread for {budget_s:.0f} s each ({wall:.1f} s wall): "
                   f"{plies} MCTS plies at {sims} sims from the GPU run's timed-window start positions (C oracle "
                   f"search) + the {predicts} policy-value forwards of the nodes they created (torch fp32 CPU); "
                   f"{procs} = the job's CPU share of the {aff} CPUs in the affinity mask"),
        "runs": runs,
    }


def measure(eng, steps, warmup, burn_in, ws, ex=None):
    """Burn-in plies (no PV forward), `warmup` untimed steps, then EXACTLY `steps`
    timed steps bracketed by barrier + synchronize, MAX over ranks.  A step = every
    slot plays plies_per_step plies, then the PV forward of every node created,
    then (N > 1) the record exchange."""
    def barrier():
        if ws > 1:
            dist.barrier()

    def step():
        eng.launch_search()
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        eng.launch_pv()
        ev[1].record()
        ctr = eng.d_counters.clone()  # per-step counters, stays on the device
        tst = None
        if eng.tree:  # list sizes of the incremental forward (device copy, no sync)
            tst = torch.zeros(8, dtype=torch.int32, device="cuda")
            _lib.check(eng.lib.gz_pv_tree_stats(ptr(eng.d_tree_ws), eng.leaf_cap, ptr(tst), stream()),
                       "gz_pv_tree_stats")
            # [6:8] = the residual-conv MFMA tile-taps the incremental kernels executed
            _lib.check(eng.lib.gz_pv_tree_exec_tiles(ptr(eng.d_tree_ws), eng.leaf_cap, ptr(tst[6:]), stream()),
                       "gz_pv_tree_exec_tiles")
        if ex is not None:
            ex.push(eng.d_records, eng.d_counters[0:4].view(torch.int32))
            ex.exchange()
        return ev, ctr, tst

    if burn_in:
        eng.advance(burn_in)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    boards0, gids0 = eng.boards()  # timed-window start positions (for the CPU baseline)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    recs = [step() for _ in range(steps)]
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    ctrs = [np.frombuffer(c.cpu().numpy().tobytes(), COUNTER_DTYPE)[0] for _, c, _ in recs]
    tree = [[int(x) for x in t.cpu()] for _, _, t in recs] if eng.tree else None
    moves = torch.tensor([float(sum(int(c["moves"]) for c in ctrs)), float(sum(int(c["mcts_moves"]) for c in ctrs))],
                         dtype=torch.float64, device="cuda")
    if ws > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(moves, op=dist.ReduceOp.SUM)
    T = float(elapsed.item())
    leaves = [min(int(c["leaves"]), eng.leaf_cap) for c in ctrs]
    exec_per_board = None
    if eng.tree:
        fl, nl = eng.tree_exec_flops()
        exec_per_board = fl / max(1, nl)
    pv_ms = [a.elapsed_time(b) for (a, b), _, _ in recs]
    return {
        "T": T, "moves": float(moves[0].item()), "mcts": float(moves[1].item()),
        "pv_ms": pv_ms, "leaves": leaves, "tree": tree, "exec_per_board": exec_per_board,
        "dropped": sum(int(c["leaves_dropped"]) + max(0, int(c["leaves"]) - eng.leaf_cap) for c in ctrs),
        "boards0": boards0, "gids0": gids0,
    }


def config5(games, sims, seed, iterations=2):
    """BASELINE config 5 on one GPU: training.main's iteration (training.run_iteration:
    self-play of `games` games with the reference's default AI -- medium, `sims` sims,
    beta 0.2, planner_steps 5, PV forward on every node -- through the sync-free record
    exchange, the 35 % 8-fold augmented dataset, 2 epochs of SGD, the StepLR step),
    `iterations` times; iterations/h from the last (the first pays MIOpen's kernel
    selection)."""
    import random
    import training
    from gzero.train import DeviceTrainer
    from neural_network import GomokuModel
    random.seed(seed)
    torch.manual_seed(seed)
    model = GomokuModel(device="cuda")
    trainer = DeviceTrainer(model)
    its = []
    for it in range(1, iterations + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = training.run_iteration(model, trainer, it, games, num_simulations=sims, planner_steps=5, beta=0.2,
                                   seed=seed, verbose=False)
        torch.cuda.synchronize()
        r["iteration_s"] = time.perf_counter() - t0
        its.append(r)
    last = its[-1]
    per1024 = last["iteration_s"] * 1024.0 / games
    return {"value": round(3600.0 / last["iteration_s"], 2), "unit": "iterations/h",
            "games_per_iteration": games,
            "per_1024_games": {"iteration_s": round(per1024, 2), "iterations_per_h": round(3600.0 / per1024, 2),
                               "note": "the same iteration scaled linearly to 1,024 games (self-play, dataset and "
                                       "SGD all grow with the record count), for comparison with round 2"},
            "iteration_s": round(last["iteration_s"], 2), "selfplay_s": round(last["selfplay_s"], 2),
            "sgd_s": round(last.get("sgd_s", 0.0), 2), "sgd_parts_s": last.get("sgd_parts_s"),
            "records": last["records"],
            "samples": last.get("samples"), "moves_played": last["moves_played"],
            "first_iteration_s": round(its[0]["iteration_s"], 2),
            "workload": (f"BASELINE config 5 on 1 GPU: training.run_iteration with {games} self-play games per "
                         f"iteration ({sims} sims, medium, beta 0.2, planner_steps 5, tree PV forward on every node, "
                         "records through gzero.dist.RecordExchange; each game played once: slots idle past the "
                         "iteration's ids and are compacted), 35 % augmentation, 2 epochs of SGD "
                         "(batch 128, Adam 8e-4, clip 0.8: the whole step on the device without autograd -- conv0, "
                         "residual tower and 1x1 head convs on gz_sgd_forward/backward (f16x3 MFMA tower), FC heads + "
                         "loss and their backward on gz_sgd_fc_loss, clip + Adam on gz_adam_step), StepLR; games per "
                         "iteration "
                         "fixed by the builder (BASELINE names none); "
                         "value from the last of "
                         f"{iterations} iterations")}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n):
    """`bench.py --gpus N` (N > 1) started without torchrun's environment: run the N
    ranks as ONE child process, `python -m torch.distributed.run --nproc-per-node N`
    on 127.0.0.1, before this process touches the GPU (no exec), relay rank 0's
    JSON line to stdout and return the child's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log("self-launch: " + " ".join(cmd))
    env = dict(os.environ, GZ_BENCH_SELF_LAUNCHED="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    line = None
    for raw in proc.stdout:  # rank 0's JSON line; anything else goes to stderr
        s = raw.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        elif s:
            log(s)
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        log("self-launch: the ranks exited 0 without a JSON line")
        rc = 1
    return rc


def rank_devices(ws, stub=False):
    """Per rank: local rank, the device it ran on and that device's PCI address and
    name, gathered to every rank (all_gather_object) -- so the line shows that the
    collective backend saw N ranks on N devices."""
    me = {"rank": dist.get_rank() if ws > 1 else 0, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
          "host": os.uname().nodename}
    if stub:
        me["device"] = "cpu"
    else:
        d = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(d)
        me.update({"device": d, "name": p.name, "arch": p.gcnArchName,
                   "pci_bus_id": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"})
    if ws == 1:
        return [me]
    out = [None] * ws
    dist.all_gather_object(out, me)
    return out


def distributed_info(ws, stub=False):
    ranks = rank_devices(ws, stub)
    return {"backend": dist.get_backend() if ws > 1 else None, "world_size": ws,
            "launch": ("self-launched torch.distributed.run" if os.environ.get("GZ_BENCH_SELF_LAUNCHED")
                       else ("torchrun (external)" if ws > 1 else "single process")),
            "distinct_devices": len({(r["host"], r.get("pci_bus_id", r["device"])) for r in ranks}),
            "ranks": ranks}


def stub_main(args):
    """--stub: the multi-rank plumbing alone, no GPU (CPU tests): rendezvous, the
    per-rank device report, EXACTLY `steps` timed steps (a step = one all-reduce)
    bracketed by barriers, max over ranks, rank 0's JSON line."""
    rank, ws = gdist.init_from_env(backend=os.environ.get("GZ_DIST_BACKEND", "gloo"))
    info = distributed_info(ws, stub=True)
    if rank == args.stub_fail_rank:  # (tests: a rank that dies after the rendezvous fails the whole run)
        log(f"rank {rank}: failing on purpose (--stub-fail-rank)")
        sys.exit(3)
    x = torch.ones(1024)

    def step():
        if ws > 1:
            dist.all_reduce(x)
    for _ in range(args.warmup):
        step()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if ws > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if ws > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC + " [stub: multi-rank plumbing only, no GPU work]", "value": 0.0,
                          "unit": "moves/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(float(el.item()) / max(1, args.steps) * 1e3, 3), "stub": True,
                          "distributed": info}), flush=True)
    if ws > 1:
        dist.destroy_process_group()


def roofline_of(m, precision):
    mean_leaves = float(np.mean(m["leaves"]))
    mean_pv_s = float(np.mean(m["pv_ms"])) / 1e3
    algorithmic = mean_leaves * PV_FLOP / mean_pv_s / 1e12 if mean_pv_s > 0 else 0.0
    achieved = algorithmic
    tree = None
    if m.get("tree"):
        # roots seen, roots w/ maps, children, full, grandchildren, patch slots
        t = np.mean(np.array(m["tree"], dtype=np.float64), axis=0)
        # executed MFMA FLOP (fp32-equivalent): full-forward nodes x 267.38 MFLOP + the
        # residual-conv tile-taps the incremental kernels counted x 16 rows x 128 x 128 x 2
        # + per incremental node its conv0 tile, 1x1 heads (radius-5 square, unclipped:
        # an upper bound) and FC heads; if the kernels counted nothing, the model of
        # tree_exec_flops
        tiles = float(t[6] + t[7])
        if tiles > 0:
            executed = (t[1] + t[3]) * PV_FLOP + tiles * TILETAP_FLOP + (t[2] + t[4]) * INC_EXTRA_FLOP
        else:
            executed = m["exec_per_board"] * mean_leaves
        achieved = executed / mean_pv_s / 1e12 if mean_pv_s > 0 else 0.0
        tree = {"roots": round(float(t[1]), 1), "children_incremental": round(float(t[2]), 1),
                "grandchildren_incremental": round(float(t[4]), 1), "patches": round(float(t[5]), 1),
                "full_other": round(float(t[3]), 1),
                "child_share": round(float((t[2] + t[4]) / max(1.0, mean_leaves)), 4),
                "executed_flop_per_launch": round(float(executed), 0),
                "algorithmic_tflops_full_forward_equivalent": round(algorithmic, 3),
                "executed_tile_taps_per_launch": round(tiles, 1),
                "executed_mflop_per_child": round((executed - (t[1] + t[3]) * PV_FLOP)
                                                  / max(1.0, t[2] + t[4]) / 1e6, 2),
                "note": ("achieved = MFMA work executed / kernel time: roots and untagged nodes the full 267.38 "
                         "MFLOP; root children (pv_dg_kernel: the delta convolution, rows sorted by tap class so a "
                         "tile skips the taps none of its rows needs) and grandchildren (pv_sib_kernel) the 16-row "
                         "MFMA tile-taps their kernels counted, plus conv0 and the heads; roots and untagged nodes "
                         "bit-identical to the full forward, children and grandchildren within 2e-5")}
    traffic, _ = load_traffic(mean_leaves, "tree" if m.get("tree") else "full") if precision == "f16x3" \
        else (None, None)
    if precision == "fp32":
        peak, note = FP32_MFMA_PEAK_TFLOPS, "exact f32 MFMA (v_mfma_f32_16x16x4_f32)"
    else:
        # each algorithmic multiply of the 3x3 convs costs 3 fp16 MFMA products
        peak = F16_MFMA_PEAK_TFLOPS / 3.0
        note = ("3-term fp16 split on v_mfma_f32_16x16x32_f16 (f32 accumulate): peak = dense fp16 MFMA "
                "peak / 3 products per fp32-equivalent multiply")
    r = {
        "kernel": (f"gz_pv_forward<{precision}> (AlphaZeroGomokuNet forward"
                   + (": pv_kernel_f16x3 tower + pv_heads_kernel FC heads + pv_prior_kernel)" if precision == "f16x3"
                      else ": pv_kernel_f32 + pv_prior_kernel)")),
        "bound": "mfma",
        "achieved": round(achieved, 3),
        "peak": round(peak, 1),
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4),
        "traffic": traffic,
        "per_launch": {"boards": round(mean_leaves, 1), "flop_per_board": PV_FLOP,
                       "avg_ms": round(float(np.mean(m["pv_ms"])), 3),
                       "us_per_board": round(float(np.mean(m["pv_ms"])) * 1e3 / max(1.0, mean_leaves), 4)},
        "note": note,
    }
    if tree:
        r["kernel"] = ("gz_pv_forward_tree<f16x3> (pv_kernel_f16x3 on roots + untagged nodes, pv_dg_kernel on "
                       "root children, pv_sib_kernel on their children; pv_heads_kernel, pv_prior_kernel)")
        r["incremental"] = tree
    dominant = ("pv_dg_kernel" if tree else ("pv_kernel_f16x3" if precision == "f16x3" else "pv_kernel_f32"))
    clk = load_clock(dominant)
    if clk:  # DVFS context: the spec peak assumes 2.4 GHz; the kernel holds less under load
        r["clock"] = {"kernel": dominant, "ghz": clk["median_ghz"], "mfma_busy": clk["median_mfma_busy"],
                      "peak_at_clock": round(peak * clk["median_ghz"] / 2.4, 1),
                      "frac_at_clock": round(achieved / (peak * clk["median_ghz"] / 2.4), 4),
                      "source": clk["source"]}
    return r


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--slots", type=int, default=4096, help="concurrent games per GPU")
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--beta", type=float, default=0.0)
    ap.add_argument("--plies-per-step", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--pv-precision", default="f16x3", choices=["f16x3", "fp32"],
                    help="policy-value forward: 3-term fp16 split (f32 accumulate) or exact fp32 MFMA")
    ap.add_argument("--pv-mode", default="tree", choices=["full", "tree"],
                    help="full: one full forward per node; tree: the incremental forward (gz_pv_forward_tree): "
                         "root children as the root's pre-BN accumulators plus the convolution of their input "
                         "differences, grandchildren from their parent's squares (within 2e-5 of full)")
    ap.add_argument("--elided-warmup", type=int, default=40, help="plies before timing the prior-elided run")
    ap.add_argument("--elided-plies", type=int, default=20)
    ap.add_argument("--no-elided", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--burn-in", type=int, default=600,
                    help="plies played before the warm-up without the PV forward (the search never reads the "
                         "priors, so the moves are the same), so the timed window sees continuous refill's "
                         "steady-state mix of game plies rather than 4096 games started together")
    ap.add_argument("--planner-steps", type=int, default=0,
                    help="BG-planner plies per rollout (BASELINE config 4: 5 with --beta 0.2)")
    ap.add_argument("--config4-steps", type=int, default=20,
                    help="N = 1 secondary: BASELINE config 4 (beta 0.2, planner_steps 5) timed over this many "
                         "steps after the same burn-in (0 = skip)")
    ap.add_argument("--config5-games", type=int, default=512,
                    help="N = 1 secondary: BASELINE config 5 (training iterations/h) with this many self-play games "
                         "per iteration (0 = skip)")
    ap.add_argument("--fp32-steps", type=int, default=4,
                    help="N = 1 secondary: the exact-fp32 PV forward timed over this many steps (0 = skip)")
    ap.add_argument("--stub", action="store_true",
                    help="multi-rank plumbing only (rendezvous, device report, timing, JSON line) without a GPU")
    ap.add_argument("--stub-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # CPU test: a failing rank
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    if args.stub:
        return stub_main(args)
    rank, ws = gdist.init_from_env()
    pool = None
    procs = 0
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        # host worker processes come from a forkserver started before this process
        # touches the GPU (no process that initialised HIP forks or execs)
        import multiprocessing as mp
        procs = host_cores()[1]
        pool = mp.get_context("forkserver").Pool(procs)
        pool.map(_cpu_warm, range(procs))  # start the workers (torch imported) now
    torch.cuda.set_device(gdist.local_device())
    if ws != args.gpus and rank == 0:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={ws}; reporting n_gpus={ws}")
    dinfo = distributed_info(ws)

    sd = weights.init_state_dict(0)
    w = PVWeights(weights.pack_pv_weights(sd), precision=args.pv_precision)
    base, stride = gdist.shard_ids(rank, ws, args.slots)
    P = args.plies_per_step
    gnw = None
    if args.planner_steps or (ws == 1 and args.config4_steps):
        from gzero import planner_nets
        gnw = planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0), planner_nets.init_dqn_state(1))

    def engine(beta, planner_steps, pv, mode="full"):
        return SelfPlayEngine(n_slots=args.slots, num_simulations=args.sims, c_puct=1.6, exploration=0.05,
                              beta=beta, seed=args.seed, pv_weights=pv, plies_per_step=P,
                              game_id_base=base, game_id_stride=stride, planner_steps=planner_steps,
                              planner_difficulty="medium", gn_weights=gnw if planner_steps else None,
                              pv_mode=mode)

    eng = engine(args.beta, args.planner_steps, w, args.pv_mode if args.pv_precision == "f16x3" else "full")
    # N > 1: the per-step RCCL all-gather of finished games' (s, pi, z) records,
    # fixed-size and sync-free (gzero.dist.RecordExchange: counts stay on the device)
    # each push copies at most 2 chunks of rows (steady state: about one record per slot
    # and ply); a burst past that is counted in record_exchange.overflow
    ex = gdist.RecordExchange(eng.record_cap, 2 * args.slots * P, "cuda", max_push=4 * args.slots * P) \
        if ws > 1 else None
    burn_in = args.burn_in
    m = measure(eng, args.steps, args.warmup, burn_in, ws, ex)
    T = m["T"]
    value = m["moves"] / T
    half = args.steps // 2
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "moves/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(T / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.pv_precision == "fp32" else (
                "f16x3 (fp32-equivalent split, f32 accumulate)"
                + ("; tree forward: root children as a delta of the root's fp32 accumulators, within 2e-5 of the "
                   "full forward and 1e-4 of the reference (tests/test_gpu_pvdelta.py)" if eng.tree else "")),
            "data": "synthetic: self-play from the empty board with random-init weights (numpy default_rng(0))",
            "config": {
                "workload": (f"BASELINE config {4 if args.planner_steps else 2}: {args.slots} concurrent self-play "
                             f"games per GPU, 15x15, {args.sims} sims/move, medium (c_puct 1.6, exploration 0.05), "
                             f"beta={args.beta}, planner_steps={args.planner_steps}, continuous refill (timed after "
                             f"{burn_in} burn-in plies: the steady-state mix of game plies); policy-value "
                             "forward + masked prior on every non-terminal node the searches create "
                             f"(reference-work mode, {args.pv_precision}"
                             + (", incremental forward of root children (delta of the root's accumulators) and "
                                "grandchildren: within 2e-5 of the full forward" if eng.tree else "")
                             + ")"),
                "pv_mode": args.pv_mode if eng.tree else "full",
                "games_per_gpu": args.slots,
                "global_games": args.slots * ws,
                "sims_per_move": args.sims,
                "plies_per_step": P,
                "burn_in_plies": burn_in,
                "parallelism": f"dp{ws} (games sharded by id, all-gather of records)",
                "pv_boards_per_step": round(float(np.mean(m["leaves"])), 1),
                "pv_boards_per_step_halves": [round(float(np.mean(m["leaves"][:half])), 1),
                                              round(float(np.mean(m["leaves"][half:])), 1)] if half else None,
                "pv_boards_dropped": m["dropped"],
            },
            "roofline": roofline_of(m, args.pv_precision),
            "mcts_moves": {"value": round(m["mcts"] / T, 3), "unit": "moves/s",
                           "share": round(m["mcts"] / m["moves"], 4) if m["moves"] else None,
                           "note": "plies decided by a search (SURVEY 8d): value counts every ply, incl. the opening "
                                   "plies 0-5 that _opening_move plays without one (ai_agent.py:138-166)"},
            "distributed": dinfo,
        }
    if ex is not None:  # every rank's leftover / lost records (a collective: all ranks take part)
        mine = torch.stack([ex.pending().reshape(()).to(torch.int64), ex.overflow.reshape(()).to(torch.int64)])
        every = torch.zeros(ws * 2, dtype=torch.int64, device=mine.device)
        dist.all_gather_into_tensor(every, mine)
        every = every.view(ws, 2).cpu().tolist()
        if rank == 0:
            out["record_exchange"] = {
                "chunk_records": ex.chunk, "bytes_per_rank_per_step": ex.chunk * ex.item,
                "pending_after": [p for p, _ in every], "overflow": [o for _, o in every],
                "note": "per rank (index = rank): records still queued after the window and records lost to "
                        "a full outbox; fixed-size RCCL all_gather_into_tensor per step, counts on the device"}
    boards0, gids0 = m["boards0"], m["gids0"]
    del eng

    # ---- N = 1 secondaries: config 4 and the exact-fp32 forward (same burn-in)
    if ws == 1 and args.config4_steps and not args.planner_steps:
        e4 = engine(0.2, 5, w, args.pv_mode if args.pv_precision == "f16x3" else "full")
        m4 = measure(e4, args.config4_steps, 2, burn_in, 1)
        gs = e4.gn_stats()
        out["config4"] = {
            "value": round(m4["moves"] / m4["T"], 3), "unit": "moves/s", "steps": args.config4_steps, "warmup": 2,
            "ms_per_step": round(m4["T"] / args.config4_steps * 1e3, 3),
            "pv_boards_per_step": round(float(np.mean(m4["leaves"])), 1),
            "pv_mode": args.pv_mode if e4.tree else "full",
            "planner_net_rows": {"full_forward": gs["full"], "incremental": gs["incremental"],
                                 "note": "GraphNet rows over the warm-up and timed steps: incremental = boards one "
                                         "stone from kept maps (the search root's, or the rollout's previous "
                                         "planner ply), bit-identical to the full forward (gn_inc_kernel)"},
            "workload": (f"BASELINE config 4: {args.slots} games, {args.sims} sims/move, beta 0.2, planner_steps 5 "
                         "(every rollout starts with 5 BGPlannerAI plies: GraphNet + OpponentDQN forward, knowledge "
                         f"search, top-k compose), PV forward + prior on every node; burn-in {burn_in} plies "
                         "searched without planner plies (the planner pipeline needs the GN forward per ply)"),
        }
        del e4
    if ws == 1 and args.fp32_steps and args.pv_precision == "f16x3" and not args.planner_steps:
        w32 = PVWeights(weights.pack_pv_weights(sd), precision="fp32")
        e32 = engine(args.beta, 0, w32)
        m32 = measure(e32, args.fp32_steps, 1, burn_in, 1)
        out["fp32"] = {"value": round(m32["moves"] / m32["T"], 3), "unit": "moves/s", "steps": args.fp32_steps,
                       "warmup": 1, "ms_per_step": round(m32["T"] / args.fp32_steps * 1e3, 3),
                       "roofline": roofline_of(m32, "fp32"),
                       "note": "config 2 with the exact-f32 MFMA forward (v_mfma_f32_16x16x4_f32)"}
        del e32, w32

    # ---- N = 1 secondary: config 5 (training iterations per hour)
    if ws == 1 and args.config5_games and not args.planner_steps:
        out["config5"] = config5(args.config5_games, args.sims, args.seed)

    # ---- prior-elided run (same kernel, no PV gather / forward)
    if not args.no_elided and not args.planner_steps:
        el = SelfPlayEngine(n_slots=args.slots, num_simulations=args.sims, c_puct=1.6, exploration=0.05,
                            beta=args.beta, seed=args.seed, pv_weights=None, plies_per_step=10,
                            game_id_base=base, game_id_stride=stride)
        done = 0
        while done < args.elided_warmup:
            n = min(10, args.elided_warmup - done)
            el.launch_search(n)
            done += n
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        e0 = time.perf_counter()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        mv_el = 0
        done = 0
        while done < args.elided_plies:
            n = min(10, args.elided_plies - done)
            el.launch_search(n)
            mv_el += int(el.counters()["moves"])
            done += n
        ev1.record()
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        e1 = torch.tensor([time.perf_counter() - e0], dtype=torch.float64, device="cuda")
        mv_t = torch.tensor([float(mv_el)], dtype=torch.float64, device="cuda")
        if ws > 1:
            dist.all_reduce(e1, op=dist.ReduceOp.MAX)
            dist.all_reduce(mv_t, op=dist.ReduceOp.SUM)
        if rank == 0:
            out["prior_elided"] = {
                "value": round(float(mv_t.item()) / float(e1.item()), 3),
                "unit": "moves/s",
                "window": f"plies {args.elided_warmup}..{args.elided_warmup + args.elided_plies} of every slot",
                "kernel_ms": round(ev0.elapsed_time(ev1), 3),
                "note": "identical moves and tuples; the reference never reads the priors (ai_agent.py:523)",
            }

    if pool is not None:
        pos = [(boards0["black"][i], boards0["white"][i], int(boards0["n_moves"][i]), int(boards0["player"][i]),
                int(gids0[i])) for i in range(min(64, len(boards0))) if boards0["n_moves"][i] >= 6]
        out["cpu_baseline"] = cpu_baseline(pool, procs, pos, args.sims, args.seed, args.cpu_seconds)
        pool.close()
        pool.join()

    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
