"""Streams with a hardware queue of their own (include/orb_abi.h orb_stream_create_dedicated).

HIP shares its GPU_MAX_HW_QUEUES hardware queues (4 by default) between plain streams
round-robin, so a caller that overlaps H2D copies, extraction and D2H copies on three plain
streams can find a copy stream on the extraction stream's queue, serialised behind it.  The
library's dedicated streams do not share a queue, whatever GPU_MAX_HW_QUEUES says.
"""
from __future__ import annotations

import ctypes

from ._native import check, hip_lib


_alive = []  # every stream handed out, kept for the life of the process (as torch's own stream pool)


def dedicated_stream(device: int = 0):
    """A torch.cuda.ExternalStream over a new dedicated-queue HIP stream on `device`.

    The HIP stream lives until the process exits (never destroyed here): torch's caching
    allocator keeps blocks allocated on a stream tied to its handle, and destroying the stream
    under them ends in a use-after-free at the allocator's next pass (bench.py crashed at exit
    that way).  C callers pair orb_stream_create_dedicated with orb_stream_destroy themselves."""
    import torch

    with torch.cuda.device(device):
        h = ctypes.c_void_p()
        check(hip_lib().orb_stream_create_dedicated(ctypes.byref(h)))
    s = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", device))
    _alive.append(s)
    return s
