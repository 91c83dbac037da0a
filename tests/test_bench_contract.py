"""bench.py's launch contract on the host (no GPU): `--gpus N` must run N ranks.

A rank whose WORLD_SIZE disagrees with --gpus exits non-zero before touching
the GPU; a plain `--gpus N` (no WORLD_SIZE) hands over to torch.distributed.run
with N ranks of the same command line (tests/test_gpu_full_size.py runs it for
real on the GPU box).
"""
import importlib.util
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mismatched_world_size_fails():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=3" in r.stderr


def test_gpus_flag_relaunches(monkeypatch):
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    import subprocess as sp

    monkeypatch.setattr(sp, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 7  # the child's exit code
    else:
        raise AssertionError("bench.main() did not exit with the launcher's code")
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]
