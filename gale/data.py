"""Synthetic InstObj traffic (the reference's producers are external; README.md:22-27 documents
the record shape ``{"instances": [[[[...]]]]}``).

Images are uniform [0, 1) floats (normalised pixels) of the model's input shape, encoded with
Java ``Float.toString`` formatting by the native encoder (what a Jackson-based producer would
emit), one or more images per record.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from gale._native import native


def synthetic_images(n: int, shape: Sequence[int], seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.random((n,) + tuple(shape), dtype=np.float32)


def encode_records(images: np.ndarray, images_per_record: int = 1) -> List[bytes]:
    """[N, H, W, C] fp32 -> list of InstObj JSON records (bytes)."""
    C = native()
    out = []
    for i in range(0, images.shape[0], images_per_record):
        out.append(C.encode_instances(np.ascontiguousarray(images[i:i + images_per_record])))
    return out


def encode_batches(records: Sequence[bytes], records_per_batch: int = 64) -> List[bytes]:
    """Group records into Kafka RecordBatch v2 blobs (for the broker's shared-append preload)."""
    K = native().kafka
    return [K.encode_batch([(None, r, -1, None) for r in records[i:i + records_per_batch]], 0, 0)
            for i in range(0, len(records), records_per_batch)]


def preload(broker, topic: str, partition: int, batches: Sequence[bytes], total_records: int,
            records_per_batch: int) -> Tuple[int, int]:
    """Append ``total_records`` records to (topic, partition) by cycling through ``batches``
    (each appended by reference). Returns (first offset, records appended)."""
    first = None
    n = 0
    i = 0
    while n < total_records:
        off = broker.append_batch_repeated(topic, partition, batches[i % len(batches)], 1)
        first = off if first is None else first
        n += records_per_batch
        i += 1
    return first, n
