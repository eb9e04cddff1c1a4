"""bench.py --gpus N starts its N ranks itself (CPU test of the launcher's argument and env handling).

The driver may call ``python bench.py --gpus N`` without an external launcher; the reference's own
multi-GPU entry point spawns its ranks the same way (mp.spawn(..., nprocs=cfg.num_gpus),
argus/train.py:373-376). Here the launcher runs a probe script in place of bench.py's body (the
body needs a GPU), over the real torch.distributed.run and a gloo rendezvous on 127.0.0.1."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

import bench


def test_needs_launch_only_without_a_launcher():
    assert bench.needs_launch(2, {})
    assert bench.needs_launch(8, {"RANK": "0"})
    assert not bench.needs_launch(1, {})
    assert not bench.needs_launch(2, {"WORLD_SIZE": "2"})
    assert not bench.needs_launch(8, {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"})


def test_launcher_argv_keeps_the_arguments_and_rendezvous():
    argv = bench.launcher_argv(4, 29555, ["--gpus", "4", "--steps", "3", "--warmup", "1"])
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in argv and "--nnodes=1" in argv
    assert "--master-addr=127.0.0.1" in argv and "--master-port=29555" in argv
    i = next(k for k, a in enumerate(argv) if a.endswith("bench.py"))
    assert argv[i + 1:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]


def test_check_world_rejects_a_mismatch():
    bench.check_world(1, 1)
    bench.check_world(8, 8)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1)
    with pytest.raises(SystemExit):
        bench.check_world(1, 2)


def test_launch_starts_n_ranks_with_the_env(tmp_path):
    probe = tmp_path / "probe.py"
    probe.write_text(textwrap.dedent("""
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        rec = {"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
               "local": int(os.environ["LOCAL_RANK"]), "dist_world": dist.get_world_size(),
               "argv": sys.argv[1:], "ipc": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}
        out = os.path.join(os.path.dirname(__file__), f"rank{rec['rank']}.json")
        open(out, "w").write(json.dumps(rec))
        dist.destroy_process_group()
    """))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = subprocess.call([sys.executable, "-c",
                            "import sys, bench; sys.exit(bench.launch(2, ['--gpus', '2', '--steps', '2'], sys.argv[1]))",
                            str(probe)], env=env, cwd=os.path.dirname(bench.__file__), timeout=180)
    assert code == 0
    recs = sorted((json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(2)), key=lambda d: d["rank"])
    assert [d["rank"] for d in recs] == [0, 1] and [d["local"] for d in recs] == [0, 1]
    for d in recs:
        assert d["world"] == 2 and d["dist_world"] == 2
        assert d["argv"] == ["--gpus", "2", "--steps", "2"]
        assert d["ipc"] == "0"
