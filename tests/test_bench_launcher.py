"""bench.py's own multi-rank launch (`python bench.py --gpus N` without torchrun): the
environment every rank receives, rank 0's JSON line relayed by the parent, and a failing rank
ending the job instead of leaving the others in a collective.  CPU only: the child script
here is a stand-in that reports its environment (and, for the gloo case, joins a real
process group and all-gathers its rank)."""
import json
import os
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

CHILD = textwrap.dedent("""
    import json, os, sys
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "REIDMI_BENCH_CHILD")
    env = {k: os.environ.get(k) for k in keys}
    if "--fail-rank" in sys.argv and os.environ["RANK"] == sys.argv[sys.argv.index("--fail-rank") + 1]:
        sys.exit(3)
    if "--gloo" in sys.argv:
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        out = [torch.zeros(1) for _ in range(dist.get_world_size())]
        dist.all_gather(out, torch.tensor([float(dist.get_rank())]))
        env["gathered"] = [float(o) for o in out]
        dist.destroy_process_group()
    elif "--fail-rank" in sys.argv:
        import time
        time.sleep(600)  # the survivors would wait in a collective: the parent must end them
    print("rank log line")
    print(json.dumps(env))
""")


def test_rank_envs():
    envs = bench.rank_envs(4, 29517, base={"PATH": "/bin", "OMP_NUM_THREADS": "16"})
    assert len(envs) == 4
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29517"
        assert e["PATH"] == "/bin" and e["OMP_NUM_THREADS"] == "16"


def test_parse_defaults_single_gpu():
    a = bench._parse([])
    assert a.gpus == 1 and a.backend == "nccl" and a.batch == 20480


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_launch_relays_rank0_line(tmp_path, capfd):
    code = bench.launch_ranks(3, ["--gloo"], script=_child(tmp_path))
    out, err = capfd.readouterr()
    assert code == 0
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    env = json.loads(lines[0])
    assert env["RANK"] == "0" and env["WORLD_SIZE"] == "3" and env["MASTER_ADDR"] == "127.0.0.1"
    assert env["REIDMI_BENCH_CHILD"] == "1"
    assert env["gathered"] == [0.0, 1.0, 2.0]
    assert "rank log line" in err  # rank 0's non-JSON output goes to stderr


@pytest.mark.parametrize("bad", ["0", "1"])
def test_launch_failing_rank_ends_job(tmp_path, bad):
    import time
    t = time.perf_counter()
    code = bench.launch_ranks(2, ["--fail-rank", bad], script=_child(tmp_path))
    assert code == 3
    assert time.perf_counter() - t < 60


def test_terminated_launcher_ends_its_ranks(tmp_path):
    """SIGTERM to the launching process (a driver's time limit) must not leave ranks behind."""
    import signal
    import subprocess
    import time
    pidfile = tmp_path / "pids"
    child = tmp_path / "child.py"
    child.write_text("import os, sys, time\n"
                     f"open({str(pidfile)!r}, 'a').write(str(os.getpid()) + '\\n')\n"
                     "time.sleep(600)\n")
    parent = subprocess.Popen([sys.executable, "-c",
                               f"import sys; sys.path.insert(0, {REPO!r}); import bench; "
                               f"sys.exit(bench.launch_ranks(2, [], script={str(child)!r}))"])
    t = time.time()
    while (not pidfile.exists() or len(pidfile.read_text().split()) < 2) and time.time() - t < 60:
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 2
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(timeout=60) != 0
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank process {pid} outlived its launcher")
