"""GPU: the C-ABI's RCCL exchange steps (csrc/comm.hip) on a one-rank
communicator — the host binding path a non-Python host uses instead of
torch.distributed: the unique id, a collective init,
C1/C3 all-gather (rank-major copy at world 1) for every dtype, C2 min/max
(identity at world 1, negation round trip exact incl. +-inf and -0.0), and
destroy. Multi-rank RCCL needs one GPU per rank; the multi-rank exchange
logic is covered by the gloo tests (tests/test_distributed.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_one_rank_comm_roundtrip(device):
    from src import _hrec

    uid = _hrec.Comm.unique_id()
    assert len(uid) == 128
    c = _hrec.Comm(0, 1, uid)
    try:
        for dt in (torch.float32, torch.float64, torch.int32, torch.int64, torch.uint8):
            x = (torch.arange(1000, device=device) * 3 % 251).to(dt)
            got = c.allgather(x)
            torch.cuda.synchronize()
            assert got.shape == (1, 1000) and torch.equal(got[0], x)
        mm = torch.tensor([[[1.5, float("inf"), -2.0], [3.0, -float("inf"), -0.0]],
                           [[-7.0, 0.25, float("inf")], [9.0, 0.5, -float("inf")]]], device=device)
        ref = mm.clone()
        c.allreduce_minmax(mm)
        torch.cuda.synchronize()
        assert torch.equal(mm, ref) and torch.equal(torch.signbit(mm), torch.signbit(ref))
    finally:
        c.close()
