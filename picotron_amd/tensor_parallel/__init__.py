from . import tensor_parallel, tp_communications  # noqa: F401
