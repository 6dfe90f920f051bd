"""bench.py's algorithmic-work figures and CLI defaults."""

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)  # defines functions only; main() runs under __main__
    return m


def test_env_step_algorithmic_bytes():
    b = _bench()
    # state r+w 2*(51*12*4 + 7*4), action 8, obs 15*4*4, reward 4, flags 2, episode stats 8
    assert b.algorithmic_bytes_per_env_step(51, 15, 4) == 5214
    assert b.algorithmic_bytes_per_env_step(51, 30, 4) == 5214 + 4 * 15 * 4


def test_minibatch_step_flops():
    b = _bench()
    S, H = 60, 256
    W = S * H + 3 * H * H + 3 * H  # matrix parameters of ActorCritic
    assert W == 212736
    assert b.ppo_flops_per_sample(S, H) == 6 * W
    assert b.ppo_flops_per_sample(S, H) * 4096 == 5228199936


def test_cli_defaults(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert (a.gpus, a.steps, a.warmup, a.config, a.hidden, a.epochs, a.minibatches) == \
        (1, 20, 5, 1, 256, 8, 32)
    # the reward-faithful recipe is the default line: 4,096-row minibatches
    assert b.CONFIGS[1] == dict(envs=4096, obs=15, order="sorted", pe="none", d=0, rollout=32)


def test_config_table_matches_baseline_json():
    """--config N is BASELINE.json's configs[N] per GPU (configs[3]: 65536 / 8 GPUs)."""
    import json

    b = _bench()
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert "4096" in cfgs[1] and b.CONFIGS[1]["envs"] == 4096
    assert "16384" in cfgs[2] and "30 vehicles" in cfgs[2] and "RoPE" in cfgs[2]
    assert (b.CONFIGS[2]["envs"], b.CONFIGS[2]["obs"], b.CONFIGS[2]["pe"]) == (16384, 30, "rope")
    assert "65536" in cfgs[3] and b.CONFIGS[3]["envs"] * 8 == 65536
    assert "32768" in cfgs[4] and (b.CONFIGS[4]["envs"], b.CONFIGS[4]["obs"]) == (32768, 30)


def test_cpu_share_is_bounded_by_the_machine():
    b = _bench()
    c = b.cpu_share()
    assert 1 <= c["share"] <= c["os_cpu_count"] and c["affinity"] <= c["os_cpu_count"]


def test_metric_string_is_baselines():
    """configs[1]'s line carries BASELINE.json's metric verbatim; other configs name their own
    workload (no 4096 x 15 text on a 32,768-env line)."""
    import json

    b = _bench()
    assert b.BASELINE_METRIC == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def test_per_kernel_roofline_reproduces_from_the_cited_rocprof_file():
    """The line's per-kernel roofline from the committed rocprofv3 summary of its workload
    (bench.rocprof_per_kernel): the four kernels parse, and their summed
    durations reproduce, within 2 %, the epoch-event step time that the same profiled command
    printed (bench_prof_c1.json: the bench line of the rocprofv3 run the summary comes from)."""
    import json
    import os

    import bench

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    line = json.loads(open(os.path.join(root, "profiles", "r6", "measure", "bench_prof_c1.json"))
                      .read().strip().splitlines()[-1])
    roof = line["roofline"]
    kf = bench.ppo_kernel_flops_per_sample(60, 256)
    got = bench.rocprof_per_kernel((1, 4096, 32, 256, "none", "sorted"), kf,
                                   roof["rows_per_launch"], roof["avg_launch_us"])
    assert got is not None and got["source"].endswith("kernel_stats_c1.txt")
    assert all(got[k]["us"] > 0 for k in ("ppo_rows", "ppo_wgrad", "ppo_wsum", "ppo_adam"))
    assert abs(got["sum_us"] / roof["avg_launch_us"] - 1.0) < 0.02
    # no summary of an unmeasured workload
    assert bench.rocprof_per_kernel((3, 8192, 128, 256, "none", "sorted"), kf, 1, 1.0) is None
    assert bench.rocprof_per_kernel((1, 4096, 32, 256, "rope", "shuffled"), kf, 1, 1.0) is None
