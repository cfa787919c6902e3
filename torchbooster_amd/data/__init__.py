"""Data sources: synthetic datasets, LMDB-backed datasets, pinned prefetcher."""
def make_named_dataset(name, root, split, **kwargs):
    return None
