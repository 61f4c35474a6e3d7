"""Host side of query deadlines: the C form of the query carries QueryContext.getEndTimeMs (pgpu_query.end_time_ms,
ABI version 2) and PGPU_ERR_TIMEOUT maps to QueryTimeoutError.  The device behaviour is in test_timeout_gpu.py."""
import ctypes
import time

from pinot_amd import _lib as L
from pinot_amd.query import QueryContext


def test_query_struct_carries_end_time():
    assert ctypes.sizeof(L.QueryC) == 64
    assert L.QueryC.end_time_ms.offset == 56
    q = QueryContext(["a"], [("COUNT", "*")])
    c, _ = q.to_c({"a": 0})
    assert c.end_time_ms == 0
    q.set_timeout(250)
    c, _ = q.to_c({"a": 0})  # the cached C form is refreshed
    now = int(time.time() * 1000)
    assert now - 50 <= c.end_time_ms - 250 <= now + 5
    q.set_timeout(None)
    assert q.to_c({"a": 0})[0].end_time_ms == 0


def test_timeout_status_maps_to_exception():
    assert L.PGPU_ERR_TIMEOUT == -7
    assert issubclass(L.QueryTimeoutError, L.PinotGpuError)
