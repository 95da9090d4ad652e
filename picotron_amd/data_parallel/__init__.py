from . import bucket, data_parallel  # noqa: F401
