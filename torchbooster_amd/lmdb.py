"""LMDB reader (reference: /root/reference/torchbooster/lmdb.py) — placeholder, replaced below."""
class LMDBReader:
    def __init__(self, path, map_size=1024 ** 4, max_readers=126):
        self.path, self.map_size, self.max_readers = path, map_size, max_readers
        self.env, self.length = None, None
