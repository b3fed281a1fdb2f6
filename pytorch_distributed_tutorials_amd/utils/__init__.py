from .checkpoint import load_checkpoint, portable_state_dict, save_checkpoint  # noqa: F401
from .env import DistEnv, dist_env  # noqa: F401
from .seed import set_random_seeds  # noqa: F401
