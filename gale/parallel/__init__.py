"""gale parallelism: data-parallel replicas, RCCL weight broadcast, partition assignment."""
