"""bench.py's latency phase joins the producer's append log with the engine's ack log
(gale/metrics.py): every acknowledged record is matched to the appended batch that holds its
offset, per partition; offsets outside the log are skipped; the stage split adds up."""

import numpy as np

from gale.metrics import append_to_ack_us, latency_stages_us


def _logs():
    # append log: (partition, base offset, records, t_ns)
    app = (np.array([0, 0, 1]), np.array([0, 10, 0]), np.array([10, 10, 5]),
           np.array([1000, 2000, 1500]))
    # ack log: (partition, offset, t_ack, t_fetch, t_take, t_done); p1/7 was never appended
    ack = (np.array([0, 0, 1, 1]), np.array([3, 15, 4, 7]), np.array([5000, 9000, 4500, 8000]),
           np.array([3000, 4000, 2500, 0]), np.array([3500, 5000, 3000, 0]),
           np.array([4000, 8000, 4000, 0]))
    return app, ack


def test_append_to_ack_join():
    app, ack = _logs()
    lat, when = append_to_ack_us(app, ack, with_ack_time=True)
    assert sorted(lat.tolist()) == [3.0, 4.0, 7.0]
    assert sorted(when.tolist()) == [4500, 5000, 9000]


def test_stage_split_sums_to_latency():
    app, ack = _logs()
    st = latency_stages_us(app, ack)
    total = st["broker_source"] + st["queue"] + st["replica"] + st["sink"]
    assert sorted(total.tolist()) == sorted(append_to_ack_us(app, ack).tolist())
    assert (st["broker_source"] >= 0).all() and (st["sink"] >= 0).all()


def test_join_is_vectorised_at_scale():
    rng = np.random.default_rng(0)
    n_batches, rpb = 20000, 16
    parts = rng.integers(0, 12, n_batches)
    base = np.zeros(n_batches, dtype=np.int64)
    nxt = np.zeros(12, dtype=np.int64)
    for i, p in enumerate(parts):
        base[i] = nxt[p]
        nxt[p] += rpb
    t_app = np.arange(n_batches, dtype=np.int64) * 1000
    app = (parts, base, np.full(n_batches, rpb), t_app)
    rec_b = np.repeat(np.arange(n_batches), rpb)
    offs = base[rec_b] + np.tile(np.arange(rpb), n_batches)
    d = rng.integers(100_000, 5_000_000, len(rec_b))
    ack = (parts[rec_b], offs, t_app[rec_b] + d, t_app[rec_b] + d // 4, t_app[rec_b] + d // 2,
           t_app[rec_b] + 3 * d // 4)
    lat = append_to_ack_us(app, ack)
    assert len(lat) == len(rec_b)
    assert np.allclose(np.sort(lat), np.sort(d / 1e3))


def test_stage_split_with_ready_time():
    """A 7-column ack log (t_ready: handed to the batcher) splits queue into ingest + batching."""
    app, ack = _logs()
    ack = ack + (np.array([3200, 4500, 2800, 0]),)
    st = latency_stages_us(app, ack)
    assert np.allclose(st["ingest"] + st["batching"], st["queue"])
    assert sorted(st["ingest"].tolist()) == [0.2, 0.3, 0.5]
