"""Runs the calibration kernels (known bytes) and 40 hwy_step launches in one process, for
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/calib/pmc_step.sh, tools/pmc_workload.sh).
The workload is bench.py's --config (env PMC_CONFIG, default 1: 4096 envs x 15 observed, sorted;
2: 16384 envs x 30 observed, shuffled + RoPE d 4; 4: 32768 envs x 30 observed, sorted), built
through the reference's make_env exactly as bench.py builds it."""
import ctypes, os, sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "highway-rope-ppo_amd"))
import torch
from bench import CONFIGS
from config.base_config import HIGHWAY_CONFIG
from experiments.config import Condition
from experiments.wrappers import make_env

wl = CONFIGS[int(os.environ.get("PMC_CONFIG", "1"))]
E = wl["envs"]
NF = 13  # state fields read and written per step (include/hwy.h)
lib = ctypes.CDLL(os.path.join(HERE, "libpmc_calib.so"))
lib.calib_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_long,
                          ctypes.c_void_p]
buf = torch.zeros(NF * E * 64, dtype=torch.int32, device="cuda:0")
sink = torch.zeros(1, dtype=torch.int32, device="cuda:0")
stream = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    assert lib.calib_run(buf.data_ptr(), sink.data_ptr(), NF, E * 64, stream) == 0
cond = {"none": Condition.SORTED if wl["order"] == "sorted" else Condition.SHUFFLED,
        "rank": Condition.SHUFFLED_RANKPE, "dist": Condition.SHUFFLED_DISTPE,
        "rope": Condition.SHUFFLED_ROPE}[wl["pe"]]
wrapped = make_env(cond, HIGHWAY_CONFIG, d_embed=wl["d"] if wl["pe"] != "none" else None,
                   env_overrides={"observation": {"vehicles_count": wl["obs"], "order": wl["order"]},
                                  "num_envs": E, "device": "cuda:0", "autoreset": True})
env = wrapped.unwrapped
env.set_seed_schedule(42)
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
for _ in range(40):
    env.step(torch.rand(E, 2, device="cuda:0", generator=g) * 0.6 - 0.3)
torch.cuda.synchronize()
print("calib bytes per launch", NF * E * 64 * 4, "envs", E, "obs", env.obs_rows, "x",
      env.obs_features, flush=True)
