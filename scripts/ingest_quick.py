"""Quick timing of the c2 ingest (bench.py's run_ingest): 5e8 ratings grouped
by user, 1M users x 100k items, int64 ids -> codes + CSR + CSC. Prints the
wall clock per ingest and per call (HIP events), and a checksum of the
outputs so variant builds (HREC_LIB) can be compared bit for bit."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "hybrid-als-twotower-recommender_amd"))
from src import _hrec  # noqa: E402

n_users, n_items = 1_000_000, 100_000
nnz_target = int(float(sys.argv[1]) if len(sys.argv) > 1 else 5e8)
g = torch.Generator(device="cuda").manual_seed(3)
counts = torch.randint(0, 2 * nnz_target // n_users + 1, (n_users,), device="cuda", generator=g)
uid = torch.repeat_interleave(torch.arange(n_users, dtype=torch.int64, device="cuda"), counts)
nnz = uid.numel()
iid = torch.randint(0, n_items, (nnz,), device="cuda", generator=g, dtype=torch.int64)
vals = torch.rand((nnz,), device="cuda", generator=g)


ORDER = os.environ.get("ORDER", "1") == "1"  # 0: the order from a separate descent pass (A/B)


def run():
    if ORDER:
        _, urow, u_ord, u_ptr = _hrec.encode_ids(uid, (0, n_users - 1), order=True)
        iu, irow, i_ord, _ = _hrec.encode_ids(iid, (0, n_items - 1), order=True)
    else:
        (_, urow), (iu, irow), u_ord, i_ord, u_ptr = (_hrec.encode_ids(uid, (0, n_users - 1)),
                                                      _hrec.encode_ids(iid, (0, n_items - 1)), None, None, None)
    a = _hrec.coo_to_csr(urow, irow, vals, n_users, alias=True, rows_in_order=u_ord, indptr=u_ptr)
    b = _hrec.coo_to_csr(irow, urow, vals, int(iu.numel()), rows_in_order=i_ord)
    return a, b


def csum(t):
    return int((t.to(torch.int64) * torch.arange(1, t.numel() + 1, device="cuda") % 1000003).sum().item()) \
        if t.dtype != torch.float32 else int((t.view(torch.int32).to(torch.int64) % 1000003).sum().item())


out = run()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    out = run()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
(a, b) = out
print(f"nnz={nnz} ingest wall ms: min {min(ts) * 1e3:.3f} median {sorted(ts)[2] * 1e3:.3f} "
      f"({36.0 * nnz / min(ts) / 8e12:.3f} of HBM at 36 B/rating)")
print("checksum", [csum(x) for x in (a[0], a[1], b[0], b[1], b[2])])
