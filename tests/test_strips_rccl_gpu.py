"""The RCCL branches of the strip exchange (config 5), executed on one GPU.

With the nccl backend (RCCL on ROCm) the strip layer does two things no gloo rehearsal reaches:

* ``StripShard.route(ops, dist)`` all-gathers the strips' count rows ON THE DEVICE with
  ``all_gather_into_tensor``, issued on the world's HIP stream (a torch ``ExternalStream``)
  between the route's kernels and its one host wait (goworld_amd/strips.py, route);
* ``exchange`` moves the halo records with ``batch_isend_irecv`` on torch's current stream,
  ordered against the world's stream by ``gwaoi_stream_before`` / ``_after`` only.

A one-rank RCCL group is legal on one GPU.  The first test runs a strip world through
``tile_tick`` (device count rows) for several ticks and checks every tick against the loopback
path (``local_tick``) on a second world and against the sequential oracle, and the gathered row
against the route's own counts.  The second test runs the exchange's P2P ordering pattern
(a buffer written by the world's stream, sent and received inside one ``batch_isend_irecv``
group, then read by the world's stream) with the rank as its own peer.

Reference: one AOI manager per space (/root/reference/engine/entity/Space.go:33,105); the strip
split itself has no reference counterpart.
"""
import os
import socket

import numpy as np
import pytest

from goworld_amd import pair_keys
from goworld_amd.strips import (HALO_WORDS, StripShard, as_words, count_row, local_tick, matrix_counts, merge_kinds,
                                 tile_tick)
from strip_scenario import D, Scenario, split_by_owner

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_one_rank():
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    if not dist.is_nccl_available():
        pytest.skip("no nccl (RCCL) backend in this torch build")
    torch.cuda.set_device(0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        yield dist
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_device_count_rows_tile_tick_match_loopback_and_oracle(oracle_mod, nccl_one_rank):
    import torch
    dist = nccl_one_rank
    seed, ticks = 13, 6
    sc_a = Scenario(n0=6000, n_strips=1, seed=seed)
    sc_b = Scenario(n0=6000, n_strips=1, seed=seed)
    A = StripShard(sc_a.max_slots, D, sc_a.edges, 0, device=0)
    B = StripShard(sc_b.max_slots, D, sc_b.edges, 0, device=0)
    ref = oracle_mod.XZList(D, sc_a.max_slots)
    try:
        for t in range(ticks):
            ta, tb = sc_a.tick(), sc_b.tick()
            oa = as_words(split_by_owner(*ta, sc_a.edges)[0], HALO_WORDS).to("cuda:0")
            ob = as_words(split_by_owner(*tb, sc_b.edges)[0], HALO_WORDS).to("cuda:0")
            send, counts, _ = tile_tick(A, dist, oa)  # device count rows: all_gather_into_tensor on RCCL
            assert A.matrix is not None and A.matrix.shape == (1, A.row_words)
            # the row RCCL gathered on the world's stream is the route's own, landed before its D2H
            np.testing.assert_array_equal(matrix_counts(A.matrix, 1)[0, :1], counts)
            want_row = count_row(counts, int(matrix_counts(A.matrix, 1)[0, 1]), A.kinds)
            np.testing.assert_array_equal(A.matrix[0], want_row, err_msg=f"tick {t}: gathered count row")
            local_tick([B], [ob])
            ea, la = A.events()
            eb, lb = B.events()
            kind, sl, nx, nz, seq, px = ta
            ref.apply(kind.astype(np.uint8), sl.astype(np.int32), nx, nz)
            oe, ol = oracle_mod.net_events(*ref.take_events())
            np.testing.assert_array_equal(np.sort(pair_keys(ea)), np.sort(pair_keys(eb)), err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(np.sort(pair_keys(la)), np.sort(pair_keys(lb)), err_msg=f"tick {t}: leaves")
            np.testing.assert_array_equal(np.sort(pair_keys(ea)), oe, err_msg=f"tick {t}: enters vs oracle")
            np.testing.assert_array_equal(np.sort(pair_keys(la)), ol, err_msg=f"tick {t}: leaves vs oracle")
            assert t == 0 or (oe.size > 0 and ol.size > 0)
    finally:
        A.close()
        B.close()


@pytest.mark.timeout(300)
def test_rccl_p2p_group_orders_against_the_world_stream(nccl_one_rank):
    """exchange's transport pattern with the rank as its own peer: the route's send buffer is
    written by the world's stream (the scatter), torch's stream waits for it without a host
    sync (gwaoi_stream_before), one batch_isend_irecv group carries it over RCCL, and the world's
    stream waits for torch's before its next kernels read the received copy (gwaoi_stream_after,
    via StripShard.finish).  The received records must be the sent ones, and the tick that
    consumes them must give the loopback tick's events."""
    import torch
    dist = nccl_one_rank
    sc_a = Scenario(n0=4000, n_strips=1, seed=29)
    sc_b = Scenario(n0=4000, n_strips=1, seed=29)
    A = StripShard(sc_a.max_slots, D, sc_a.edges, 0, device=0)
    B = StripShard(sc_b.max_slots, D, sc_b.edges, 0, device=0)
    try:
        for t in range(4):
            ta, tb = sc_a.tick(), sc_b.tick()
            oa = as_words(split_by_owner(*ta, sc_a.edges)[0], HALO_WORDS).to("cuda:0")
            ob = as_words(split_by_owner(*tb, sc_b.edges)[0], HALO_WORDS).to("cuda:0")
            send, counts, tele = A.route(oa)
            recv = torch.empty_like(send)
            tele_r = torch.empty_like(tele)
            ops = [dist.P2POp(dist.isend, send, 0), dist.P2POp(dist.irecv, recv, 0)]
            if tele.shape[0]:
                ops += [dist.P2POp(dist.isend, tele, 0), dist.P2POp(dist.irecv, tele_r, 0)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            # the received copy replaces the local slice: same records, other buffer
            k = A.kinds  # this receiver's statistics: its own route's, for destination 0
            A.finish(recv, send[:0], tele_r, kinds=merge_kinds([(k[0][0], k[1][0], k[2][0])]))
            local_tick([B], [ob])
            ea, la = A.events()
            eb, lb = B.events()
            assert torch.equal(recv, send) and torch.equal(tele_r, tele), f"tick {t}: P2P payload"
            np.testing.assert_array_equal(np.sort(pair_keys(ea)), np.sort(pair_keys(eb)), err_msg=f"tick {t}: enters")
            np.testing.assert_array_equal(np.sort(pair_keys(la)), np.sort(pair_keys(lb)), err_msg=f"tick {t}: leaves")
    finally:
        A.close()
        B.close()
