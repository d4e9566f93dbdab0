"""ldt_amd — MI355X-native batch decode for Lance/Arrow image batches.

Drop-in for lance-distributed-training's hot path:

    from ldt_amd import decode_tensor_image, collate_fn          # lance_iterable.py:38, lance_map_style.py:21
    from ldt_amd import LanceDataset, SafeLanceDataset, get_safe_loader
    from ldt_amd import ShardedBatchSampler, ShardedFragmentSampler, FullScanSampler

All decode/resize/shard arithmetic runs in libldt.so's gfx950 HIP kernels.
"""
from ._lib import ImageDecodeError, LdtError, load_library, version  # noqa: F401
from .dataset import (ArrowDataset, LanceDataset, SafeLanceDataset, dataset,  # noqa: F401
                      get_safe_loader, write_dataset)
from .sampler import DistributedSampler, FullScanSampler, ShardedBatchSampler, ShardedFragmentSampler  # noqa: F401
from .transforms import (IMAGENET_MEAN, IMAGENET_STD, PROGRESSIVE_DEPTH, DecodePipeline, ResidentBatch, bind_numa, collate_fn,  # noqa: F401
                         decode_arrow, decode_tensor_image, make_collate_fn, make_to_tensor_fn,
                         register_host, resize_raw, unregister_host)

__version__ = "0.1.0"
