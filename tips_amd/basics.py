"""Lifecycle — mirrors tips/tensorflow/basics.py:5-31 (TipsBasics) over libtips_hip.so.

Differences from the reference, on purpose:
  * init is lazy (first size()/rank()/allreduce call, or an explicit init()),
    not at import, so importing the package never touches a GPU;
  * `initialized()` calls the exported `tips_is_initialize` (the reference's
    basics.py:25 calls a misspelled `tips_is_initialized`);
  * when torch.distributed is already initialised with world_size > 1, the
    RCCL unique id is handed out through it instead of the library's own TCP
    bootstrap (tips_init reads RANK / WORLD_SIZE / MASTER_ADDR itself).
"""
import atexit
import ctypes
import os
import threading

from . import _lib

_init_lock = threading.Lock()
_atexit_registered = False


def _torch_dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    force = os.environ.get("TIPS_BOOTSTRAP", "") == "torch"  # use the group even at world size 1
    if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or force):
        return dist
    return None


def share_unique_id(dist, make_id):
    """Rank 0's make_id() bytes, delivered to every rank of the torch.distributed group."""
    payload = [make_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(payload, src=0)
    return payload[0]


class TipsBasics(object):
    """Wrapper class for the basic TiPS APIs (basics.py:5-31)."""

    def __init__(self, pkg_path=None):
        self.CORE_CTYPES = _lib.lib() if pkg_path is None else ctypes.CDLL(pkg_path, mode=ctypes.RTLD_GLOBAL)

    def init(self):
        """Initialise TiPS (collective over all ranks). Idempotent."""
        global _atexit_registered
        L = self.CORE_CTYPES
        with _init_lock:
            if L.tips_is_initialize():
                return
            dist = _torch_dist()
            if dist is not None:
                rank, size = dist.get_rank(), dist.get_world_size()
                nbytes = L.tips_unique_id_bytes()

                def make_id():
                    buf = ctypes.create_string_buffer(nbytes)
                    _lib.check("tips_get_unique_id", L.tips_get_unique_id(buf, nbytes))
                    return buf.raw

                idbuf = ctypes.create_string_buffer(share_unique_id(dist, make_id), nbytes)
                _lib.check("tips_init_rank", L.tips_init_rank(rank, size, -1, idbuf, nbytes))
            else:
                L.tips_init()
                if not L.tips_is_initialize():
                    raise _lib.TipsError("tips_init", -2, _lib.last_error())
            if not _atexit_registered:
                atexit.register(self.shutdown)
                _atexit_registered = True

    def shutdown(self):
        """Shut down the TiPS service (basics.py:20-22)."""
        self.CORE_CTYPES.tips_shutdown()

    def initialized(self):
        return bool(self.CORE_CTYPES.tips_is_initialize())

    def size(self):
        self.init()
        return self.CORE_CTYPES.tips_size()

    def rank(self):
        self.init()
        return self.CORE_CTYPES.tips_rank()


_basics = None


def basics():
    global _basics
    if _basics is None:
        _basics = TipsBasics()
    return _basics


def init():
    basics().init()


def shutdown():
    basics().shutdown()


def is_initialized():
    return basics().initialized()


def size():
    return basics().size()


def rank():
    return basics().rank()
