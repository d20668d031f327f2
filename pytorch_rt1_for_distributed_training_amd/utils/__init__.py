"""Checkpointing, logging, profiling helpers."""
from .checkpoint import (ModelCheckpoint, build_checkpoint, load_checkpoint, load_model_state,  # noqa: F401
                         save_checkpoint)
from .logging import CSVLogger, MultiLogger, TensorBoardLogger  # noqa: F401
