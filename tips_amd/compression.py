"""Gradient compression — mirrors tips/tensorflow/compression.py:20-75.

Compression.fp16 is usable here: the device path has an fp16 allreduce
(dtype code 4), whereas the reference casts to tf.float16 and then hits the
op's {int32, int64, float32, float64} constraint (ops.cc:121).
"""
import numpy as np

from . import tensors


class Compressor(object):
    """Interface for compressing and decompressing a given tensor (compression.py:20-31)."""

    @staticmethod
    def compress(tensor):
        pass

    @staticmethod
    def decompress(tensor, ctx):
        pass


class NoneCompressor(Compressor):
    """Default no-op compression (compression.py:34-46)."""

    @staticmethod
    def compress(tensor):
        return tensor, None

    @staticmethod
    def decompress(tensor, ctx):
        return tensor


def _is_floating(t):
    if tensors.is_torch(t):
        return t.dtype.is_floating_point
    return np.issubdtype(np.asarray(t).dtype, np.floating)


class FP16Compressor(Compressor):
    """Cast floating tensors to 16-bit for the wire (compression.py:49-66)."""

    @staticmethod
    def compress(tensor):
        compressed = tensor
        if _is_floating(tensor):
            if tensors.is_torch(tensor):
                import torch
                compressed = tensor.to(torch.float16)
            else:
                compressed = np.asarray(tensor).astype(np.float16)
        return compressed, tensor.dtype

    @staticmethod
    def decompress(tensor, ctx):
        if ctx is None or not _is_floating(tensor):
            return tensor
        if tensors.is_torch(tensor):
            return tensor.to(ctx)
        return np.asarray(tensor).astype(ctx)


class Compression(object):
    """Optional gradient compression algorithm used during allreduce (compression.py:69-75)."""
    none = NoneCompressor
    fp16 = FP16Compressor
