"""Training engine: fused step, flat Adam, LR schedule, Lightning-style trainer loop."""
from .optim import FlatAdam, multistep_lr  # noqa: F401
from .step import TrainEngine, split_batch, to_device  # noqa: F401
