"""Launcher + fault tolerance: a rank is killed by
the fault-injection hook mid-run, the launcher reports it, restarts the pod,
and training resumes from the last complete checkpoint to the end."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "fleetx_amd", "configs", "nlp", "gpt", "pretrain_gpt_345M_single_card.yaml")


def _train_args(out):
    ov = ["Model.hidden_size=64", "Model.num_layers=2", "Model.num_attention_heads=4",
          "Model.vocab_size=256", "Model.max_position_embeddings=64", "Global.device=cpu",
          "Global.local_batch_size=2", "Global.micro_batch_size=2", "Global.global_batch_size=None",
          "Engine.max_steps=6", "Engine.logging_freq=1", "Engine.eval_freq=1000",
          "Engine.save_load.save_steps=2", "Engine.save_load.output_dir=%s" % out,
          "Data.Train.dataset.name=SyntheticGPTDataset", "Data.Train.dataset.max_seq_len=32",
          "Data.Train.dataset.vocab_size=256", "Data.Train.loader.num_workers=0",
          "Data.Eval.dataset.name=SyntheticGPTDataset", "Data.Eval.dataset.max_seq_len=32",
          "Data.Eval.dataset.vocab_size=256", "Data.Eval.loader.num_workers=0"]
    args = [os.path.join(ROOT, "tools", "train.py"), "-c", CFG]
    for o in ov:
        args += ["-o", o]
    return args


def _env(**kw):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **kw)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_launcher_restarts_failed_pod_and_resumes(tmp_path):
    log_dir = tmp_path / "log"
    cmd = [sys.executable, "-m", "fleetx_amd.launch", "--nproc_per_node", "2",
           "--log_dir", str(log_dir), "--max_restart", "1"] + _train_args(tmp_path / "out")
    # rank 1 dies after finishing step 3 (the step-2 checkpoint exists by then)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=_env(FLEETX_FAULT_INJECT="1:3"))
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "Pod failed" in r.stdout and "rank 1, exit code 17" in r.stdout
    assert "restarting pod (1/1)" in r.stdout
    log0 = (log_dir / "workerlog.0").read_text()
    log1 = (log_dir / "workerlog.1").read_text()
    assert "fault injection" in log1
    second = log0.split("==== launch attempt 1")[1]
    assert "Load checkpoint from" in second and "epoch_0_step_2" in second
    assert "batch: 3," in second and "batch: 6," in second and "batch: 2," not in second
    assert "training finished" in second


def test_launcher_gives_up_after_max_restart(tmp_path):
    cmd = [sys.executable, "-m", "fleetx_amd.launch", "--nproc_per_node", "1",
           "--log_dir", str(tmp_path / "log"), "--max_restart", "0",
           os.path.join(ROOT, "tools", "train.py"), "-c", "/nonexistent.yaml"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=_env())
    assert r.returncode != 0
    assert "Pod failed" in r.stdout and "rank 0" in r.stdout


def test_child_env_contract():
    from fleetx_amd import launch as L
    a = L.parse_args(["--devices", "4,5", "--nnodes", "2", "--node_rank", "1", "x.py"])
    env = L.child_env(a, L.device_list(a), 1, 2, "10.0.0.1", 6000)
    assert env["RANK"] == "3" and env["WORLD_SIZE"] == "4" and env["LOCAL_RANK"] == "1"
    assert env["PADDLE_TRAINER_ID"] == "3" and env["PADDLE_RANK_IN_NODE"] == "1"
    assert env["FLAGS_selected_gpus"] == "5" and env["HIP_VISIBLE_DEVICES"] == "4,5"
    assert env["FLEETX_RESTART_COUNT"] == "2" and env["MASTER_PORT"] == "6000"


def test_bench_graph_capture_stays_in_warmup():
    """bench.py's whole-step graph: on by default for one GPU only when the
    warmup covers the capture step (the engine runs GRAPH_EAGER_STEPS eager
    steps, then captures), so a capture never lands in the timed region;
    multi-rank runs stay eager; --hip-graph forces either way."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    import inspect
    eager = inspect.signature(EagerEngine._fit_graphed).parameters["warmup"].default
    assert bench.GRAPH_EAGER_STEPS == eager
    assert bench.use_graph(-1, 1, eager + 1) == 1
    assert bench.use_graph(-1, 1, eager) == 0
    assert bench.use_graph(-1, 2, 10) == 0
    assert bench.use_graph(0, 1, 10) == 0
    assert bench.use_graph(1, 1, 0) == 1
