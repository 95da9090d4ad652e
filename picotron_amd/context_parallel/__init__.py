from . import context_parallel, cp_communications  # noqa: F401
