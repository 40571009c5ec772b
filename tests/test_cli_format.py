"""Golden-format tests of the reference console output and result files (SURVEY §2.5, §4 layer 6).

Runs the 13-argument CLI end to end on a tiny synthetic dataset written in the reference
text layout and checks every console line against the reference templates
(ref src/naive.py:86,93,156,198,209; :407) and the ``%5.3f`` result files (ref src/util.py:32-36).
"""
import os
import re

import numpy as np
import pytest

from erasurehead_amd.cli import main as cli_main
from erasurehead_amd.data.synthetic import generate_to_disk, synthetic_dir

LOGISTIC_LINE = re.compile(r"^Iteration (\d+): Train Loss = [ \d.]{5,}, Test Loss = [ \d.]{5,}, AUC = [ \d.]{5,}, "
                           r"Total time taken =[ \d.]{5,}$")
LINEAR_LINE = re.compile(r"^Iteration (\d+): Train Loss = \d+\.\d{6}, Test Loss = \d+\.\d{6}, Total time taken =[ \d.]{5,}$")


def _data(root, n_procs=5, n=200, d=6, partial=(0, 0, 0)):
    s, P, part = partial
    out, parts = synthetic_dir(root, n_procs, n, d, s, P, part)
    generate_to_disk(n, d, parts, out, rng=np.random.RandomState(0), verbose=False)
    return out


@pytest.mark.parametrize("args,prefix", [
    (("0", "1", "0", "0", "0"), "naive_acc_"),
    (("1", "1", "0", "0", "0"), "coded_acc_1_"),
    (("1", "1", "0", "1", "0"), "replication_acc_1_"),
    (("1", "1", "0", "2", "0"), "avoidstragg_acc_1_"),
    (("1", "1", "0", "3", "3"), "replication_acc_1_"),  # AGC collides with replication (ref quirk)
])
def test_console_and_files(args, prefix, tmp_path, capsys):
    root = str(tmp_path) + "/"
    ddir = _data(root)
    is_coded, s, P, ver, k = args
    rc = cli_main(["5", "200", "6", root, "0", "artificial", is_coded, s, P, ver, k, "0", "GD", "--num-itrs", "12",
                   "--device", "cpu", "--seed", "1"])
    assert rc == 0
    lines = capsys.readouterr().out.splitlines()
    assert lines[0].startswith("---- Starting ")
    assert lines[1] == "\t >>> At Iteration 0" and "\t >>> At Iteration 10" in lines
    tot = [l for l in lines if l.startswith("Total Time Elapsed: ")]
    assert len(tot) == 1 and re.match(r"^Total Time Elapsed: \d+\.\d{3}$", tot[0])
    its = [l for l in lines if l.startswith("Iteration ")]
    assert [int(LOGISTIC_LINE.match(l).group(1)) for l in its] == list(range(12))
    loaded = [l for l in lines if l.startswith(">> Loaded ")]
    if prefix.startswith(("naive", "coded")):  # ref naive.py:160-164: partitions 1..W-1 (the off-by-one)
        assert loaded == [">> Loaded %d" % j for j in range(1, 4)]
        assert lines.index(tot[0]) < lines.index(loaded[0]) < lines.index(its[0])
    else:
        assert loaded == []
    assert lines[-1] == ">>> Done"
    res = os.path.join(ddir, "results")
    for kind in ("training_loss", "testing_loss", "auc", "timeset"):
        body = open(os.path.join(res, prefix + kind + ".dat")).read().splitlines()
        assert len(body) == 12
        assert all(re.match(r"^ ?-?\d+\.\d{3} $", l) for l in body), body[:2]
    wt = np.loadtxt(os.path.join(res, prefix + "worker_timeset.dat"))
    assert wt.shape == (12, 4)


def test_least_squares_console(tmp_path, capsys):
    root = str(tmp_path) + "/"
    _data(root)
    rc = cli_main(["5", "200", "6", root, "0", "artificial", "0", "0", "0", "0", "0", "0", "GD", "--num-itrs", "3",
                   "--device", "cpu", "--loss", "least_squares", "--lr", "0.01"])
    assert rc == 0
    its = [l for l in capsys.readouterr().out.splitlines() if l.startswith("Iteration ")]
    assert len(its) == 3 and all(LINEAR_LINE.match(l) for l in its), its


def test_usage_and_rejections(tmp_path, capsys):
    assert cli_main(["1", "2"]) == 0
    assert capsys.readouterr().out.startswith("Usage: python main.py")
    root = str(tmp_path) + "/"
    _data(root, n_procs=9)
    # FRC with W % (s+1) != 0 prints the reference error and exits cleanly
    assert cli_main(["9", "200", "6", root, "0", "x", "1", "2", "0", "1", "0", "0", "GD", "--device", "cpu"]) == 0
    assert "Error: n_workers must be multiple of n_stragglers+1!" in capsys.readouterr().out


def test_lr_schedules():
    from erasurehead_amd.config import RunConfig

    c = RunConfig(3, 10, 2, "/tmp", num_itrs=4)
    np.testing.assert_allclose(c.eta(), [10.0] * 4)
    c = RunConfig(3, 10, 2, "/tmp", num_itrs=4, lr_kind="invscaling")  # ref main.py:42-44
    np.testing.assert_allclose(c.eta(), [10.0 * 90.0 / (i + 90.0) for i in range(1, 5)])
    c = RunConfig(3, 10, 2, "/tmp", num_itrs=4, lr=0.1, lr_kind="exponential")  # ref main.py:46
    np.testing.assert_allclose(c.eta(), [0.1 * 0.98 ** i for i in range(1, 5)])


def test_extension_flags_parse_and_run(tmp_path, capsys):
    """--share-partitions / --device-loop reach RunConfig; shared partitions train identically."""
    from erasurehead_amd.cli import parse

    cfg, _ = parse(["5", "200", "6", "/d/", "0", "artificial", "1", "1", "0", "1", "0", "0", "GD",
                    "--share-partitions", "--device-loop", "graph"])
    assert cfg.share_partitions and cfg.device_loop == "graph"
    cfg, _ = parse(["5", "200", "6", "/d/", "0", "artificial", "1", "1", "0", "1", "0", "0", "GD"])
    assert not cfg.share_partitions and cfg.device_loop == "auto"
    root = str(tmp_path) + "/"
    _data(root)
    outs = []
    for extra in ([], ["--share-partitions"]):
        assert cli_main(["5", "200", "6", root, "0", "artificial", "1", "1", "0", "1", "0", "0", "GD",
                         "--num-itrs", "4", "--seed", "3", *extra]) == 0
        outs.append([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("Iteration")])
    strip = [[ln.split(", Total time")[0] for ln in o] for o in outs]
    assert strip[0] == strip[1] and len(strip[0]) == 4


def test_main_gpus_flag_launches_ranks(tmp_path):
    """`python main.py <13 args> --gpus 2` starts two ranks from one command (CPU / gloo here) and
    prints the reference console lines once (rank 0)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = str(tmp_path) + "/"
    r = subprocess.run([sys.executable, os.path.join(root, "main.py"), "5", "2000", "20", out, "0", "synthetic", "1", "1",
                        "0", "3", "2", "0", "AGD", "--data", "synthetic", "--num-itrs", "4", "--seed", "0",
                        "--gpus", "2"], cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert sum(l.startswith("Iteration ") and "Train Loss" in l for l in r.stdout.splitlines()) == 4
