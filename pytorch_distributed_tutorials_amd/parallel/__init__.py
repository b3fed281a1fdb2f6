from .buckets import ddp_bucket_plan, plan_buckets  # noqa: F401
from .comm import backend_name, destroy, init_distributed, native_comm, rank, world_size  # noqa: F401
from .ddp import DistributedDataParallel  # noqa: F401
from .flat import FlatParamSpace, flatten_buffers  # noqa: F401
