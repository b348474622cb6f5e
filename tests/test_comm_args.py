"""CPU checks of the C-ABI communicator (kanode_comm_*): argument validation runs before any RCCL or
device call, and failures without a communicator leave their message in kanode_comm_last_error(NULL)."""
import ctypes as C

import pytest

import kanode
from kanode import _lib as L
from kanode import comm


def test_comm_create_rejects_bad_ranks_and_ids():
    for nranks, rank in ((0, 0), (2, 2), (2, -1)):
        with pytest.raises(kanode.KanodeError, match="rank"):
            comm.Comm(nranks, rank, bytes(L.COMM_ID_BYTES))
    with pytest.raises(ValueError):
        comm.Comm(1, 0, bytes(16))
    out = C.c_void_p()
    assert L.lib().kanode_comm_create(1, 0, None, 0, C.byref(out)) == 1
    assert b"id is NULL" in L.lib().kanode_comm_last_error(None)
    assert out.value is None


def test_comm_null_communicator():
    assert L.lib().kanode_comm_allreduce_sum(None, None, 0, 1, None) == 1
    assert b"null communicator" in L.lib().kanode_comm_last_error(None)
    assert L.lib().kanode_comm_size(None) == -1 and L.lib().kanode_comm_rank(None) == -1
    L.lib().kanode_comm_destroy(None)   # no-op
