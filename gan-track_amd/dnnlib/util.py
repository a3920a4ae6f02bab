"""Subset of SG3/dnnlib/util.py the training path uses: EasyDict (:33-51), Logger (:56-100),
class-name resolution (:260-316) and formatting helpers.  No URL fetching (open_url is absent on
purpose: the reference's network fetches are out of scope and unavailable offline)."""
import importlib
import os
import sys
import types


class EasyDict(dict):
    """dict with attribute access (SG3 dnnlib/util.py:33-51)."""

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value

    def __delattr__(self, name):
        del self[name]


class Logger:
    """Tee stdout/stderr into a file (SG3 dnnlib/util.py:56-100)."""

    def __init__(self, file_name=None, file_mode='w', should_flush=True):
        self.file = open(file_name, file_mode) if file_name is not None else None
        self.should_flush = should_flush
        self.stdout, self.stderr = sys.stdout, sys.stderr
        sys.stdout = sys.stderr = self

    def write(self, text):
        if isinstance(text, bytes):
            text = text.decode()
        if not text:
            return
        if self.file is not None:
            self.file.write(text)
        self.stdout.write(text)
        if self.should_flush:
            self.flush()

    def flush(self):
        if self.file is not None:
            self.file.flush()
        self.stdout.flush()

    def close(self):
        self.flush()
        if sys.stdout is self:
            sys.stdout = self.stdout
        if sys.stderr is self:
            sys.stderr = self.stderr
        if self.file is not None:
            self.file.close()
            self.file = None


def format_time(seconds):
    s = int(round(seconds))
    if s < 60:
        return f'{s}s'
    if s < 3600:
        return f'{s // 60}m {s % 60:02d}s'
    if s < 86400:
        return f'{s // 3600}h {(s // 60) % 60:02d}m {s % 60:02d}s'
    return f'{s // 86400}d {(s // 3600) % 24:02d}h {(s // 60) % 60:02d}m'


def make_cache_dir_path(*paths):
    base = os.environ.get('DNNLIB_CACHE_DIR') or os.path.join(os.path.expanduser('~'), '.cache', 'dnnlib')
    return os.path.join(base, *paths)


def get_obj_by_name(name):
    """'pkg.mod.Attr' -> object; the longest importable module prefix wins (SG3 util.py:260-305)."""
    parts = name.split('.')
    for i in range(len(parts) - 1, 0, -1):
        mod_name = '.'.join(parts[:i])
        try:
            obj = importlib.import_module(mod_name)
        except ModuleNotFoundError:
            continue
        for attr in parts[i:]:
            obj = getattr(obj, attr)
        return obj
    return importlib.import_module(name)


def call_func_by_name(*args, func_name=None, **kwargs):
    assert func_name is not None
    fn = get_obj_by_name(func_name)
    assert callable(fn)
    return fn(*args, **kwargs)


def construct_class_by_name(*args, class_name=None, **kwargs):
    """SG3 dnnlib/util.py:314-316."""
    return call_func_by_name(*args, func_name=class_name, **kwargs)


def get_module_from_obj_name(name):
    parts = name.split('.')
    for i in range(len(parts) - 1, 0, -1):
        try:
            return importlib.import_module('.'.join(parts[:i])), '.'.join(parts[i:])
        except ModuleNotFoundError:
            continue
    raise ModuleNotFoundError(name)


def is_top_level_function(obj):
    return callable(obj) and isinstance(obj, types.FunctionType) and obj.__name__ in sys.modules[obj.__module__].__dict__
