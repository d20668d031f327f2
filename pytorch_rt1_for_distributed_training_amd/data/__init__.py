"""Input pipeline: synthetic windows, Language-Table episode windows, device prefetch."""
from .episodes import (DecodeAndRandomResizedCrop, EpisodeWindowDataset, collate_fn,  # noqa: F401
                       convert_reference_episodes, make_fake_episodes, write_episode)
from .prefetch import DevicePrefetcher  # noqa: F401
from .synthetic import SyntheticDataset, SyntheticStream, make_batch  # noqa: F401
from .shards import ShardBatchLoader, decode_on_device, is_shard, pack_shard  # noqa: F401
