"""bench.py's multi-rank launch on the host (no GPU): `python bench.py --gpus N` starts the N ranks
itself through torchrun (the reference's launch, train.py:2 / template/base_job.slurm:64), refuses a
launcher whose WORLD_SIZE disagrees with --gpus, and forwards rank 0's one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_command_line():
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2", "--backend", "nccl"]
    cmd = bench.launcher_cmd(argv, 8, 29611)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29611" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv                   # the script's own arguments pass through unchanged


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_mismatched_world_size_is_refused():
    """torchrun with 2 ranks but --gpus 8: exit non-zero before touching the GPU."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, env=_env(WORLD_SIZE="2", RANK="0"), timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_launch_forwards_one_result_line(monkeypatch, tmp_path, capsys):
    """launch_ranks runs the job as a child and forwards only rank 0's JSON line to stdout."""
    fake = tmp_path / "fake_ranks.py"
    fake.write_text("import json\nprint('RCCL version banner')\n"
                    "print(json.dumps({'metric': 'm', 'value': 1.0, 'n_gpus': 2, 'ranks': 2}))\n"
                    "print('trailing noise')\n")
    monkeypatch.setattr(bench, "launcher_cmd", lambda argv, n, port: [sys.executable, str(fake)])
    assert bench.launch_ranks(["--gpus", "2"], 2) == 0
    out = capsys.readouterr()
    lines = out.out.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2
    assert "RCCL version banner" in out.err and "trailing noise" in out.err


def test_launch_without_result_fails(monkeypatch, tmp_path):
    fake = tmp_path / "crash.py"
    fake.write_text("import sys\nsys.exit(3)\n")
    monkeypatch.setattr(bench, "launcher_cmd", lambda argv, n, port: [sys.executable, str(fake)])
    assert bench.launch_ranks(["--gpus", "2"], 2) == 3
    fake.write_text("print('no json')\n")
    assert bench.launch_ranks(["--gpus", "2"], 2) == 1


@pytest.mark.gpu
def test_gloo_rehearsal_two_ranks_one_line():
    """The one-GPU rehearsal of the driver's N = 2 run: both ranks on cuda:0 over gloo, DP over a
    2-layer model; one JSON line reporting 2 GPUs and 2 ranks."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--layers", "2", "--grad-acc", "2", "--steps", "1", "--warmup", "1", "--no-probe"],
                       capture_output=True, text=True, env=_env(), timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == 2 and d["backend"] == "gloo"
    assert d["config"]["parallelism"] == "dp2"


def test_synthetic_loader_fresh_batches():
    """bench.py's loader draws a new step's tokens after each pass (fresh=True; the first pass is the
    replaying loader's), so its final_loss is not a memorisation curve; fresh=False replays."""
    import torch
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.train import SyntheticMicroBatchDataLoader
    pgm.setup_process_group_manager(1, 1, 1, 1)
    a = SyntheticMicroBatchDataLoader(2, 16, 3, 100, torch.device("cpu"), seed=5)
    b = SyntheticMicroBatchDataLoader(2, 16, 3, 100, torch.device("cpu"), seed=5, fresh=True)
    first_a = [next(a)["input_ids"].clone() for _ in range(3)]
    first_b = [next(b) for _ in range(3)]
    assert all(torch.equal(x, y["input_ids"]) for x, y in zip(first_a, first_b))
    second_a = [next(a)["input_ids"] for _ in range(3)]
    second_b = [next(b) for _ in range(3)]
    assert all(torch.equal(x, y) for x, y in zip(first_a, second_a))
    assert not any(torch.equal(x, y["input_ids"]) for x, y in zip(first_a, second_b))
    for y in second_b:   # targets stay the inputs shifted by one
        assert y["input_ids"].shape == (2, 16) and torch.equal(y["input_ids"][:, 1:], y["target_ids"][:, :-1])
        assert int(y["input_ids"].max()) < 100


def test_bench_assembles_the_8_rank_dp2_tp2_pp2_grid_on_cpu():
    """`bench.py --gpus 8 --backend gloo --assemble-only`: the driver's 8-GPU grids are built before
    any GPU run -- here config 4's dp2 tp2 pp2 (process_group_manager.py:13's view(dp, pp, cp, tp)):
    every grid coordinate once, each pipeline stage's shard the same size on all of its ranks, the
    stages' layers covering the model, the embedding on stage 0 and the lm_head on the last stage."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--backend", "gloo",
           "--assemble-only", "--tp", "2", "--pp", "2", "--layers", "2", "--seq", "256"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(OMP_NUM_THREADS="1"))
    if r.returncode != 0 and "Signal 6 (SIGABRT)" in r.stderr:
        # once in ~15 runs one of the 8 gloo ranks on this 8-CPU container has died of SIGABRT inside
        # the gloo transport during rendezvous (not reproduced in isolation); one fresh launch
        sys.stderr.write(r.stderr[-3000:])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["assembled"] and d["ranks"] == 8 and d["config"]["parallelism"] == "dp2-pp2-tp2"
    for e in d["per_rank"]:
        dp_, pp_, cp_, tp_ = e["grid"]
        assert e["rank"] == ((dp_ * 2 + pp_) * 1 + cp_) * 2 + tp_
        assert e["embedding"] == (pp_ == 0) and e["lm_head"] == (pp_ == 1)
        assert e["layers"] == ([0] if pp_ == 0 else [1]) and e["buckets"] > 0


def test_pmc_kernel_key_for_dual_labels():
    """bench.py's roofline names the dominant kernel by its GemmProbe label; the PMC traffic file keys
    kernels by rocprofv3 name + workgroup count: the dual launches map onto gemm_8ph_dual_kernel with
    one workgroup per 256x256 tile (the split-K dX halves counted twice)."""
    k = bench.pmc_kernel_key
    assert k("dual dX 4096x2048x16384 e2 + dW 16384x2048x4096 e1") == \
        "void gemm_8ph_dual_kernel<true, false, 2, false, false, 1> [768 WG]"     # gate|up dX halves + dW
    assert k("dual dX 4096x2048x6144 e2 + dW 6144x2048x4096,2048x2048x4096 e1") == \
        "void gemm_8ph_dual_kernel<true, false, 2, false, false, 1> [512 WG]"     # q|k|v halves + q|k|v, o dW
    assert k("dual dX 4096x8192x2048 e6 + dW 2048x8192x4096 e3") == \
        "void gemm_8ph_dual_kernel<true, false, 6, false, false, 3> [768 WG]"     # down dX + SwiGLU bwd + dW
    assert k("linear_wgrad_grouped") == "linear_wgrad_grouped"


def test_resolve_batch_defaults():
    """Config 2's mbs 4 x grad_acc 32 by default; pure TP (config 3) mbs 32 x grad_acc 4 -- the same
    128 sequences per step -- unless either is given; cp / pp keep the config-2 defaults."""
    import bench

    def r(*a):
        x = bench.resolve_batch(bench.build_parser().parse_args(list(a)))
        return x.mbs, x.grad_acc
    assert r() == (4, 32)
    assert r("--tp", "8") == (32, 4) and r("--tp-proxy", "8") == (32, 4)
    assert r("--tp", "8", "--mbs", "4") == (4, 32) and r("--tp", "8", "--grad-acc", "4") == (4, 4)
    assert r("--model", "llama2-7b", "--tp", "2", "--pp", "2", "--gpus", "8") == (4, 32)
    assert r("--cp", "8", "--mbs", "1") == (1, 32)
