"""Config plumbing mirroring SG3/dnnlib (EasyDict, construct_class_by_name)."""
from .util import EasyDict, make_cache_dir_path  # noqa: F401
