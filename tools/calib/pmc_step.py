"""Runs the calibration kernels (known bytes) and 40 hwy_step launches in one process, for
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/calib/pmc_step.sh)."""
import ctypes, os, sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "highway-rope-ppo_amd"))
import torch
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

E = 4096
NF = 13  # state fields read and written per step (include/hwy.h)
lib = ctypes.CDLL(os.path.join(HERE, "libpmc_calib.so"))
lib.calib_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_long,
                          ctypes.c_void_p]
buf = torch.zeros(NF * E * 64, dtype=torch.int32, device="cuda:0")
sink = torch.zeros(1, dtype=torch.int32, device="cuda:0")
stream = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    assert lib.calib_run(buf.data_ptr(), sink.data_ptr(), NF, E * 64, stream) == 0
env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
for _ in range(40):
    env.step(torch.rand(E, 2, device="cuda:0", generator=g) * 0.6 - 0.3)
torch.cuda.synchronize()
print("calib bytes per launch", NF * E * 64 * 4)
