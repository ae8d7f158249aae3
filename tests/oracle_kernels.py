"""A CPU kernel provider backed by the oracle -- TEST INFRASTRUCTURE ONLY.

It has the interface of deepep_amd.kernels.HipKernels and is injected by the CPU
tests into ElasticBuffer (`buffer._kernels = OracleKernels()`) to exercise the host
orchestration (plans, dispatch, RCCL/gloo exchange, stream bookkeeping) without a
GPU.  The product never selects it.
"""
from typing import Optional

import torch

import oracle


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class OracleKernels:
    name = 'oracle'

    def combine_reduce(self, mode, src, out, num_units, table=None, row_weights=None, bias0=None, bias1=None,
                       wtable=None, wsrc=None, out_weights=None, units_per_block=0, error_flag=None, stream=None):
        assert src.device.type == 'cpu' and out.device.type == 'cpu'
        for t in (src, out, table, row_weights, bias0, bias1, wtable, wsrc, out_weights):
            assert t is None or t.dim() == 1 or t.stride(-1) == 1
        hidden = out.shape[1]
        rc = oracle.rows_lib().oracle_combine_rows(
            mode, int(row_weights is not None),
            _p(src), src.shape[0], src.stride(0) if src.shape[0] else hidden,
            _p(table), table.stride(0) if table is not None else 0, table.shape[1] if table is not None else 1,
            _p(row_weights), _p(bias0), _p(bias1),
            _p(out), out.stride(0) if out.shape[0] else hidden, num_units, hidden,
            _p(wtable), wtable.stride(0) if wtable is not None else 0,
            _p(wsrc), _p(out_weights), out_weights.shape[1] if out_weights is not None else 0,
            out_weights.stride(0) if out_weights is not None else 0)
        assert rc == 0, 'oracle_combine_rows failed'

    def build_local_plan(self, src_metadata, num_recv_tokens, num_topk, num_max_tokens_per_rank, expanded,
                         plan, num_tokens, topk_idx=None, wtable=None, stream=None):
        meta = src_metadata[:num_recv_tokens]
        plan.fill_(-1)
        t = (meta[:, 0] % num_max_tokens_per_rank).long()
        if expanded:
            plan[t] = meta[:, 2:2 + plan.shape[1]]
        else:
            plan[t, 0] = torch.arange(num_recv_tokens, dtype=torch.int32)
        if wtable is not None:
            wtable.fill_(-1)
            inv = torch.full((num_tokens,), -1, dtype=torch.int64)
            inv[t] = torch.arange(num_recv_tokens)
            k = torch.arange(num_topk).view(1, -1)
            ok = (topk_idx >= 0) & (inv.view(-1, 1) >= 0)
            wtable.copy_(torch.where(ok, inv.view(-1, 1) * num_topk + k, torch.full_like(topk_idx, -1)).to(torch.int32))
