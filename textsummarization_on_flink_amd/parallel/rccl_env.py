"""RCCL's CU cap for every rank process (torch-free: launchers apply it before anything imports
torch or touches the GPU)."""
import os

# RCCL's CU footprint: a collective kernel runs one workgroup per channel.  Every rank process
# caps the channels (NCCL_MAX_NCHANNELS / NCCL_MAX_CTAS, set in its environment before RCCL
# initialises -- the bench launcher, the worker runtime and ``init_from_env`` all apply
# ``rccl_env``), so in-flight all-reduces hold at most this many CUs.  The persistent encoder LSTM
# needs all its workgroups resident: a launch grid leaving at least this many CUs free may share
# the GPU with RCCL (train/trainer.py; tests/test_gpu_production.py holds exactly this many CUs with
# a spinning kernel during the captured BPTT phase).  An 86 MB fp32 gradient all-reduce at 8 ranks
# moves 2 x 7/8 x 86 MB = 150 MB per rank; 64 channels spread it over all 7 xGMI links
# (~0.2-0.4 ms at 50-100 GB/s per link and direction), more channels do not add link bandwidth.
RCCL_MAX_CHANNELS = 64


def rccl_env(env=None) -> dict:
    """Cap RCCL's channels (hence CUs) in ``env`` (default: this process's environment) unless the
    user set them; returns ``env``."""
    env = os.environ if env is None else env
    env.setdefault("NCCL_MAX_NCHANNELS", str(RCCL_MAX_CHANNELS))
    env.setdefault("NCCL_MAX_CTAS", env["NCCL_MAX_NCHANNELS"])
    return env


def rccl_cu_reserve() -> int:
    """CUs an in-flight RCCL collective may hold: the effective channel cap."""
    try:
        return int(os.environ.get("NCCL_MAX_NCHANNELS", RCCL_MAX_CHANNELS))
    except ValueError:
        return RCCL_MAX_CHANNELS
