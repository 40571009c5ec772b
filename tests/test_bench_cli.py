"""bench.py launch contract: `python bench.py --gpus N` measures N ranks from one plain command
(ref run_approx_coding.sh:47-49 starts every rank with one mpirun), and a WORLD_SIZE that
disagrees with --gpus is an error, never a silently mislabelled measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--steps", "3", "--warmup", "1", "--n-rows", "2400", "--n-cols", "20", "--floor-rounds", "8"]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""  # CPU / gloo ranks
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


def test_bench_gpus3_relaunches_three_ranks(tmp_path):
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", *TINY, "--straggler-steps", "6",
                        "--json-out", str(out)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 3
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2]
    assert d["ranks"][0]["role"].startswith("master")
    assert sorted({w for x in d["ranks"] for w in x["workers"]}) == list(range(8))
    # partition shards (default on several ranks): every (worker, partition) of the W=8, s=2
    # uneven-FRC messages is computed on exactly one rank: 3*3 + 3*3 + 2*2 = 22 shards
    assert d["shard"] == "partition"
    units = [u for us in d["placement"].values() for u in us]
    assert len(units) == len(set(units)) == 22
    for r, us in d["placement"].items():  # a partition's replicas share one rank
        for u in us:
            p = u.split(":")[1]
            assert all(p not in v for rr, vs in d["placement"].items() if rr != r for v in vs)
    for x in d["ranks"]:
        assert x["transport"] == "gloo"
        assert x["local_grad_us"] > 0
    assert d["ranks"][1]["recv_beta_us"] >= 0
    assert 0 < d["fraction_of_rows_used_in_decode"] <= 1
    assert d["host_driven_ms_per_step"] > 0
    assert d["loss_target"] > 0 and d["naive_iters_to_loss_floor"] is not None
    # the reference topology (one message per rank) and the straggler sub-run, in the same JSON
    assert d["message_placement_ms_per_step"] > 0
    st = d["straggler"]
    assert st["late_rank"] == 2 and st["late_workers"] == [2, 5] and st["placement"] == "message"
    for k in ("agc_lazy", "agc_lazy_no_straggler", "naive", "naive_no_straggler"):
        assert st[k]["ms_per_step"] > 0 and [x["rank"] for x in st[k]["ranks"]] == [0, 1, 2]
    assert st["agc_lazy"]["drain"] == "lazy" and st["naive"]["drain"] == "carry"
    assert st["naive"]["round_ms_mean"] >= 5.0  # naive waits for the late rank every round
    assert st["agc_lazy_round_slowdown"] > 0 and st["naive_round_slowdown"] > 1.0
    # first contact (bench.first_contact): a bounded check run on the headline's loop before timing
    fc = d["first_contact"]
    assert fc["rounds"] == 30 and [x["ok"] for x in fc["ladder"]] == [True]
    assert fc["ladder"][0]["round_loop"] == "python" and fc["transport"] == "gloo"
    assert d["release_form"] == "n/a" and d["config"]["round_loop_reason"]


def test_bench_world8_tolerant_co_headline(tmp_path):
    """Round-5 verdict item 6: at N > 1 the JSON carries the straggler-tolerant topology as a co-headline
    (value_tolerant: message placement, the reference's one worker per process) next to `value` (partition
    shards), both timed like the headline, with the job's own scaling efficiencies against rank 0's
    single-GPU run of the same config; 8 gloo ranks (the 8-GPU code path on the CPU)."""
    out = tmp_path / "b8.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *TINY, "--no-floor",
                        "--straggler-steps", "4", "--late-ms", "2", "--json-out", str(out)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 8 and d["shard"] == "partition"
    assert d["value_tolerant"] > 0 and d["value_tolerant_placement"] == "message"
    assert d["value_tolerant"] == d["message_placement"]["ms_per_step"] / 1e3
    assert d["message_placement"]["steps"] == d["steps"]
    assert d["single_gpu_s_per_iter"] > 0
    assert d["scaling_efficiency"] == d["single_gpu_s_per_iter"] / (8 * d["value"])
    assert d["scaling_efficiency_tolerant"] == d["single_gpu_s_per_iter"] / (8 * d["value_tolerant"])
    assert set(d["scaling_placements"]) == {"value", "value_tolerant"}
    assert "agc_lazy" in d["straggler"] and d["first_contact"]["ladder"][-1]["ok"]


def test_bench_one_gpu_straggler_block(tmp_path):
    """N = 1 carries the paper's claim in the driver's own JSON: naive, AGC with the reference's drain
    and AGC with the lazy drain under Exp virtual delays, with floors and wall-clock to the common target
    (ref src/approximate_coding.py:144-158,182-183,198-205)."""
    out = tmp_path / "b1.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *TINY[:-1], "30",
                        "--straggler-mean-ms", "3", "--no-breakdown", "--clock-warmup-ms", "0",
                        "--json-out", str(out)],
                       cwd=str(tmp_path), env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    st = d["straggler_virtual"]
    assert st["rounds"] == 30 and st["delay_mean_s"] == pytest.approx(0.003)
    assert st["loss_target"] == pytest.approx(st["naive"]["final_train_loss"] * 1.01)
    for name, drain in (("naive", "carry"), ("agc_drain", "all"), ("agc_lazy", "lazy")):
        x = st[name]
        assert x["drain"] == drain
        for k in ("sum_timeset_s", "loop_wallclock_s", "floor_timeset_s", "floor_loop_s", "model_loop_s",
                  "overhead_ms_per_round", "iters_to_target", "wallclock_s_to_target", "timeset_s_to_target"):
            assert x[k] is not None, (name, k)
        # a run never beats the zero-compute replay of its own delays
        assert x["sum_timeset_s"] >= x["floor_timeset_s"] and x["loop_wallclock_s"] >= x["floor_loop_s"]
    # AGC decodes with fewer workers; the drain waits for the tail (the naive floor), lazy does not
    assert st["agc_drain"]["used_workers_per_round"] < 8 == st["naive"]["used_workers_per_round"]
    assert st["agc_drain"]["floor_loop_s"] == pytest.approx(st["naive"]["floor_loop_s"])
    assert st["agc_lazy"]["floor_loop_s"] < st["naive"]["floor_loop_s"]
    assert st["agc_lazy"]["stale_skipped"] > 0
    # the verdict fields are the JSON's own comparison of its wall clocks.  Which way it goes on this CPU
    # depends on how loaded the test machine is (the rounds' compute is host time here), so it is pinned
    # for consistency, not for its sign; the GPU records carry the claim (lazy 0.360 s vs naive 0.822 s
    # to target, profiles/round5/final/bench.json) and the floors above carry it deterministically.
    lz, nv = st["agc_lazy"]["wallclock_s_to_target"], st["naive"]["wallclock_s_to_target"]
    assert st["agc_lazy_beats_naive_to_target"] is (lz < nv)
    assert st["agc_lazy"]["speedup_to_target_vs_naive"] == pytest.approx(nv / lz)


def test_bench_subrun_failure_keeps_the_headline(tmp_path):
    """A run after the headline that fails on every rank alike (here: worker rank 1's round loop raises in
    the instrumented breakdown run, ERASUREHEAD_SABOTAGE=subrun:raise:1:2) is contained: the JSON line still
    carries the headline value, names the failed sub-run in `subrun_failures`, and the collective sub-runs
    after it are skipped on every rank (no hang, exit 0)."""
    out = tmp_path / "b.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY, "--straggler-steps", "4",
                        "--subrun-timeout", "3", "--clock-warmup-ms", "0", "--json-out", str(out)],
                       cwd=str(tmp_path), env=dict(_env(), ERASUREHEAD_SABOTAGE="subrun:raise:1:2"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["ms_per_step"] > 0
    assert list(d["subrun_failures"]) == ["breakdown"], d.get("subrun_failures")
    assert "rank 1" in d["subrun_failures"]["breakdown"] or "test hook" in d["subrun_failures"]["breakdown"]
    assert "straggler" not in d and "loss_target" not in d and "single_gpu_s_per_iter" not in d
    assert "host_driven_ms_per_step" not in d


def test_bench_world_size_mismatch_fails(tmp_path):
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY, "--no-floor"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_decode_row_fraction_counts_covered_partitions():
    """bench.py's fraction_of_rows_used_in_decode: AGC (W=8, s=2, k=6, uneven groups) stopping on
    groups {0,1,2} and {3,4,5} decodes 6 of the 8 partitions; every group covered -> 1."""
    sys.path.insert(0, ROOT)
    import bench
    from erasurehead_amd.codes import make_scheme
    from erasurehead_amd.codes.schemes import Arrival

    sch = make_scheme("approx", 8, 2, 8000, 6, 0, allow_uneven=True)
    two_groups = [(w, 0, 0.0) for w in (0, 1, 2, 3, 4, 5)]
    all_groups = [(w, 0, 0.0) for w in (0, 3, 6)]
    assert bench.decode_row_fraction(sch, [two_groups], Arrival) == 0.75
    assert bench.decode_row_fraction(sch, [all_groups], Arrival) == 1.0
    assert bench.decode_row_fraction(sch, [two_groups, all_groups], Arrival) == 0.875


@pytest.mark.gpu
def test_bench_preflight_failure_rebuilds_on_comm_path(tmp_path):
    """A failed per-pair preflight (here: worker rank 1 reports a bad payload word through the test
    hook) is a collective verdict: every rank rebuilds the trainer on the RCCL code path (loopback
    when ranks share the GPU) and the JSON records why, instead of one rank raising while the
    others wait.  2 ranks time-share the box's GPU."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", ERASUREHEAD_SABOTAGE="preflight:1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = tmp_path / "f.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY, "--no-floor",
                        "--preflight", "50", "--json-out", str(out)],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert "payload words wrong" in d["peer_preflight_failure"] and "rank 1" in d["peer_preflight_failure"]
    assert "peer_preflight" not in d
    assert all(x["transport"] == "loopback" for x in d["ranks"])
    fp = d["fallback_preflight"]  # the fallback was checked over its own path before timing
    assert [x["rank"] for x in fp] == [1] and fp[0]["payload_errors"] == 0 and fp[0]["path"] == "loopback"
    assert "same" in d["fallback_mechanism"] or "mailbox" in d["fallback_mechanism"]
    assert d["ms_per_step"] > 0


def _gpu_bench(tmp_path, name, extra_env, *args):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = tmp_path / name
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *TINY, "--no-floor",
                        "--no-straggler", "--preflight", "50", "--json-out", str(out), *args],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(out.read_text())


@pytest.mark.gpu
def test_bench_first_contact_cross_device_selection(tmp_path):
    """The first 8-GPU run's path, forced on the one-GPU box: a faked device map (two GPUs) selects the
    strict release forms, the arbiter runs (ERASUREHEAD_DEVICE_MASTER=on) and checks itself with
    integrity-tagged rounds before timing; the JSON carries the release form, the loop and why, the
    device map and the per-pair preflight round trips."""
    d = _gpu_bench(tmp_path, "x.json", dict(ERASUREHEAD_DEVICE_MASTER="on", ERASUREHEAD_FAKE_DEVICE_MAP="g0,g1"))
    assert d["release_form"] == "strict" and "different GPUs" in d["release_reason"]
    assert d["device_map"] == {"0": "fake:g0", "1": "fake:g1"}
    fc = d["first_contact"]
    assert [(x["round_loop"], x["ok"]) for x in fc["ladder"]] == [("arbiter", True)]
    assert fc["ladder"][0]["release_form"] == "strict" and fc["round_loop"] == "arbiter"
    assert d["config"]["round_loop"].startswith("device-driven (arbiter") and d["config"]["round_loop_reason"]
    assert [x["rank"] for x in d["peer_preflight"]] == [1] and d["peer_preflight"][0]["rtt_us_p50"] > 0
    assert all(x["release_form"] == "strict" for x in d["ranks"])
    assert d["ms_per_step"] > 0


@pytest.mark.gpu
def test_bench_first_contact_steps_down_on_integrity_failure(tmp_path):
    """A torn message in the first-contact check (rank 1's put of round 3 flips a byte after its
    checksum, for that check run only): the arbiter's integrity check fails the round, every rank
    agrees on the verdict, the job steps down to the native pump in the same processes, checks that,
    and times the headline on it -- the JSON says what failed and what ran."""
    d = _gpu_bench(tmp_path, "s.json", dict(ERASUREHEAD_DEVICE_MASTER="on", ERASUREHEAD_FAKE_DEVICE_MAP="g0,g1",
                                           ERASUREHEAD_SABOTAGE="firstcontact:msg:1:3"), "--selfcheck-timeout", "4",
                   "--naive")  # naive: every message enters the decode, so the torn rows are read
    fc = d["first_contact"]
    lad = fc["ladder"]
    assert [(x["round_loop"], x["ok"]) for x in lad] == [("arbiter", False), ("native pump", True)], lad
    assert "rank" in lad[0]["failure"] and "arbiter -> native pump" in lad[0]["step_down"]
    assert fc["round_loop"] == "native pump"
    assert d["config"]["round_loop"] == "host-driven (native pump)"
    assert d["ms_per_step"] > 0


def test_worker_round_start_latency_maps_both_clocks():
    """bench.worker_round_start_latency: the master's beta(i) put stamp and each worker's round-i start stamp
    live on different GPU clocks; both are mapped to the host clock through each rank's (tick0, t0, hz)
    calibration before they are subtracted, unstamped rounds (-1) are skipped, and the median over the
    rounds from ``first`` on is reported per worker rank in microseconds."""
    sys.path.insert(0, ROOT)
    from bench import worker_round_start_latency

    hz0, hz1 = 100e6, 25e6
    R = 6
    beta_put = [[-1, -1] for _ in range(R)]
    rounds = [[-1] * 10 for _ in range(R)]
    for i in range(R):
        t_put = 10.0 + i * 1e-3  # host seconds of the master's post-put stamp
        beta_put[i][1] = 5_000 + (t_put - 2.0) * hz0  # master clock: tick0 5000 at host t0 = 2.0 s
        rounds[i][9] = 700 + (t_put + (3 + i) * 1e-6 - 4.0) * hz1  # worker: starts 3 + i us later
    rounds[2][9] = -1  # an unstamped round is skipped
    recs = [{"rank": 0, "clock": (0, 5_000, 2.0, hz0), "beta_put": beta_put, "probes": []},
            {"rank": 1, "clock": (0, 700, 4.0, hz1), "rounds": rounds}]
    lat = worker_round_start_latency(recs, first=1)
    assert set(lat) == {1}
    assert abs(lat[1] - 6.5) < 0.05, lat  # rounds 1, 3, 4, 5: 4, 6, 7, 8 us -> median 6.5
