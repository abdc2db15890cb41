"""CPU: bench.py's multi-GPU entry (no GPU call happens before these points).

* `--gpus N` without a launcher (WORLD_SIZE unset) starts N rank processes
  through torch.distributed.run with the same arguments, as a child process
  whose exit status bench.py returns;
* `--config c3` (BASELINE configs[2], sized for 8 GPUs) refuses fewer ranks
  with a message naming the requirement.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_n_without_launcher_starts_the_ranks(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd, **kw: calls.append(cmd) or 7)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3", "--warmup", "2"])
    assert bench.main() == 7
    (cmd,) = calls
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "2"]


def test_c3_needs_eight_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c3"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "8-GPU configuration" in r.stderr and "--gpus 8" in r.stderr
