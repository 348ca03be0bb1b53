"""Packed state arenas (``parallel/arena.py``): layout after ``add_state`` / ``.to()``, unchanged ``state_dict``, in-place
reset, and the sync engine sending a packed bucket as one span (no ``torch.cat``) on a 2-rank gloo pool."""
import io

import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import Metric, MetricCollection
from torchmetrics_amd.parallel import arena
from tests.helpers import run_ddp


class _Rebinder(Metric):
    """Update rebinds its states (``x = x + v``): falls out of the arena on every update."""

    def __init__(self):
        super().__init__()
        self.add_state("a", torch.zeros(3), "sum")
        self.add_state("b", torch.zeros(2), "sum")

    def update(self, v):
        self.a = self.a + v
        self.b = self.b + 2 * v

    def compute(self):
        return self.a.sum() + self.b.sum()


def _data(seed=0, n=64, c=5):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, c, generator=g), torch.randint(0, c, (n,), generator=g)


def test_states_packed_after_init_and_to():
    m = tm.MulticlassStatScores(5, average=None)
    assert arena.is_packed([m])
    tp = m.tp
    assert tp.untyped_storage().data_ptr() == m.fn.untyped_storage().data_ptr()
    m = m.to(torch.float64).to("cpu")
    assert arena.is_packed([m])
    p, t = _data()
    m.update(p, t)
    assert arena.is_packed([m])  # in-place accumulation keeps the layout


def test_state_dict_round_trip_unchanged():
    p, t = _data(1)
    m = tm.MulticlassStatScores(5, average=None)
    m.persistent(True)
    m.update(p, t)
    sd = m.state_dict()
    assert set(sd) == {"tp", "fp", "tn", "fn"}
    for k, v in sd.items():
        assert torch.equal(v, getattr(m, k))
        assert v.untyped_storage().nbytes() == v.numel() * v.element_size()  # compact: not the whole arena
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    m2 = tm.MulticlassStatScores(5, average=None)
    m2.persistent(True)
    m2.load_state_dict(torch.load(buf, weights_only=True))
    for k in sd:
        assert torch.equal(getattr(m2, k), sd[k])
    assert torch.equal(m2.compute(), m.compute())


def test_reset_refills_packed_states_in_place():
    m = tm.MulticlassStatScores(5, average=None)
    p, t = _data(2)
    m.update(p, t)
    ids = [id(getattr(m, k)) for k in ("tp", "fp", "tn", "fn")]
    m.reset()
    assert [id(getattr(m, k)) for k in ("tp", "fp", "tn", "fn")] == ids
    assert all(int(getattr(m, k).sum()) == 0 for k in ("tp", "fp", "tn", "fn"))
    m.update(p, t)
    held = m.tp[1:]  # a view of the arena: reset must not clobber it
    before = held.clone()
    m.reset()
    assert torch.equal(held, before) and int(m.tp.sum()) == 0


def test_rebinding_metric_is_eventually_left_unpacked():
    m = _Rebinder()
    for i in range(arena.MAX_REPACKS + 3):
        m.update(torch.tensor(1.0))
        arena.pack([m])
    assert not arena.is_packed([m])  # gave up: its buckets use the cat path
    assert m._arena_repacks > arena.MAX_REPACKS
    m.reset()
    assert "_arena_repacks" not in m.__dict__


def test_deepcopy_keeps_layout():
    m = tm.MulticlassStatScores(5, average=None)
    c = m.clone()
    assert arena.is_packed([c])
    c.tp += 1
    assert int(m.tp.sum()) == 0


# ------------------------------------------------------------------------------------------ 2-rank gloo sync
def _body_sync_no_cat(rank, world):
    p, t = _data(10 + rank)
    m = tm.MulticlassStatScores(5, average=None)
    m.update(p, t)
    local = {k: getattr(m, k).clone() for k in ("tp", "fp", "tn", "fn")}
    calls = []
    real_cat = torch.cat

    def counting_cat(*a, **k):
        calls.append(1)
        return real_cat(*a, **k)

    torch.cat = counting_cat
    try:
        m.sync()
    finally:
        torch.cat = real_cat
    assert not calls, "a packed bucket must be sent as one span"
    for k, v in local.items():
        want = v.clone()
        torch.distributed.all_reduce(want)
        assert torch.equal(getattr(m, k), want)
    m.unsync()
    for k, v in local.items():
        assert torch.equal(getattr(m, k), v)
    assert arena.is_packed([m])


def test_sync_sends_packed_bucket_without_cat():
    run_ddp(_body_sync_no_cat)


def _body_collection_arena(rank, world):
    p, t = _data(20 + rank)
    members = {"acc": tm.MulticlassAccuracy(5), "prec": tm.MulticlassPrecision(5), "cm": tm.MulticlassConfusionMatrix(5)}
    refs = {k: m.clone() for k, m in members.items()}
    coll = MetricCollection(members, compute_groups=True)
    import torchmetrics_amd.collections as coll_mod

    real_sync, real_cat, cats = coll_mod.sync_state_dicts, torch.cat, []

    def counting_sync(*a, **k):  # torch.cat calls made by the engine itself during the collection's sync
        def cat(*ca, **ck):
            cats.append(1)
            return real_cat(*ca, **ck)

        torch.cat = cat
        try:
            return real_sync(*a, **k)
        finally:
            torch.cat = real_cat

    coll_mod.sync_state_dicts = counting_sync
    try:
        for step in range(3):
            coll.update(p, t)
            cats.clear()
            out = coll.compute()
            if step:
                assert not cats, "packed leaders: every bucket is one span"
            leaders = [getattr(coll, cg[0]) for cg in coll._groups.values()]
            assert arena.is_packed(leaders)  # every leader's sum states in one arena per dtype
            for k, m in refs.items():
                m.update(p, t)
                assert torch.allclose(out[k].float(), m.compute().float()), (step, k)
    finally:
        coll_mod.sync_state_dicts = real_sync


def test_collection_leaders_share_one_arena():
    run_ddp(_body_collection_arena)


def _body_rebinder_sync(rank, world):
    m = _Rebinder()
    for _ in range(arena.MAX_REPACKS + 3):
        m.update(torch.tensor(float(rank + 1)))
        assert float(m.compute()) == pytest.approx(21.0 * m._update_count)
    assert float(m.a[0]) == m._update_count * (rank + 1)


def test_rebinding_metric_syncs_correctly():
    run_ddp(_body_rebinder_sync)


# ------------------------------------------------------------------------------- growable arena of cat list states
class _CatMetric(Metric):
    full_state_update = False

    def __init__(self, **kw):
        super().__init__(**kw)
        self.add_state("x", [], dist_reduce_fx="cat", persistent=True)

    def update(self, v):
        self.x.append(v)

    def compute(self):
        from torchmetrics_amd.utilities.data import dim_zero_cat

        return dim_zero_cat(self.x).sum(0)


def test_cat_arena_amortised_growth_and_values():
    m = _CatMetric()
    g = torch.Generator().manual_seed(0)
    seen, caps = [], []
    for step in range(9):
        v = torch.randn(10 + step, 3, generator=g)
        seen.append(v)
        m.update(v)
        torch.testing.assert_close(m.compute(), torch.cat(seen).sum(0))
        m._computed = None
        assert len(m.x) == 1 and m.x[0].shape == (sum(s.shape[0] for s in seen), 3)
        if step:
            buf, view = m.__dict__["_cat_arenas"]["x"]
            assert view is m.x[0] and view.data_ptr() == buf.data_ptr()
            caps.append(buf.shape[0])
    assert caps[0] == 10 + 11  # first fold: exactly what it needs
    assert len(set(caps)) <= 4  # doubling: few re-allocations over 9 steps
    assert all(b >= a for a, b in zip(caps, caps[1:]))


def test_cat_arena_state_dict_pickle_reset_and_forward():
    import pickle

    m = _CatMetric()
    for i in range(3):  # folds: 10 rows (exact), then 15 rows in a 20-row buffer
        m.update(torch.full((5, 2), float(i)))
        m.compute()
        m._computed = None
    folded = m.x[0]
    assert folded.untyped_storage().nbytes() > folded.numel() * folded.element_size()  # spare capacity
    sd = m.state_dict()
    assert sd["x"][0].untyped_storage().nbytes() == sd["x"][0].numel() * sd["x"][0].element_size()
    torch.testing.assert_close(sd["x"][0], folded)
    buf = io.BytesIO()
    torch.save(sd, buf)
    assert buf.tell() < 2 * folded.numel() * folded.element_size() + 4096
    m2 = pickle.loads(pickle.dumps(m))
    assert "_cat_arenas" not in m2.__dict__
    torch.testing.assert_close(m2.compute(), m.compute())
    # forward(): the batch value uses its own plain cat, the global arena keeps growing in place
    m._computed = None
    before = m.__dict__["_cat_arenas"]["x"][0]
    out = m(torch.ones(3, 2))
    torch.testing.assert_close(out, torch.full((2,), 3.0))
    m.compute()
    assert m.__dict__["_cat_arenas"]["x"][0] is before
    m.reset()
    assert "_cat_arenas" not in m.__dict__ and m.x == []


def test_cat_arena_falls_back_for_autograd_and_mixed_shapes():
    m = _CatMetric()
    a = torch.ones(2, 3, requires_grad=True)
    m.update(a)
    m.update(torch.ones(1, 3))
    out = m.compute()
    assert out.requires_grad and "_cat_arenas" not in m.__dict__
    m2 = _CatMetric()
    m2.update(torch.ones(2, 3))
    m2.update(torch.ones(4))  # different trailing shape: plain cat semantics (here: an error, as torch.cat)
    with pytest.raises(RuntimeError):
        m2.compute()


@pytest.mark.gpu
def test_cat_arena_per_step_compute_gpu():
    """Per-step compute() of an unbinned curve metric on ROCm: the folded preds / target live in one growing HBM
    buffer and every step's value equals a fresh CPU metric over the same history."""
    g = torch.Generator().manual_seed(3)
    m = tm.classification.BinaryAUROC().cuda()
    ref = tm.classification.BinaryAUROC()
    for step in range(12):
        p, t = torch.rand(1000, generator=g), torch.randint(0, 2, (1000,), generator=g)
        m.update(p.cuda(), t.cuda())
        ref.update(p, t)
        torch.testing.assert_close(m.compute().cpu(), ref.compute(), rtol=1e-6, atol=1e-6)
        ref._computed = None
    buf, view = m.__dict__["_cat_arenas"]["preds"]
    assert buf.is_cuda and view is m.preds[0] and view.shape[0] == 12000 and buf.shape[0] >= 12000


class _ViewCompute(Metric):
    """compute() returns a VIEW of a SUM state (the case sys.getrefcount cannot see)."""

    full_state_update = False

    def __init__(self):
        super().__init__()
        self.add_state("a", torch.zeros(4), "sum")
        self.add_state("b", torch.zeros(2), "sum")

    def update(self, v):
        self.a += v
        self.b += v[:2]

    def compute(self):
        return self.a[:2]


def test_forward_does_not_mutate_held_views():
    """forward()'s in-place fold of the batch into the global SUM states must not change a previously returned
    compute() value that aliases the state, nor a user-held view of it (the reference merges out of place)."""
    m = _ViewCompute()
    m.update(torch.ones(4))
    v = m.compute()
    assert v.tolist() == [1.0, 1.0]
    m(torch.ones(4))
    assert v.tolist() == [1.0, 1.0]
    assert m.compute().tolist() == [2.0, 2.0]
    held = m.a.view(2, 2)
    m(torch.ones(4))
    assert held.flatten().tolist() == [2.0, 2.0, 2.0, 2.0]
    assert m.a.tolist() == [3.0] * 4
    # nothing held any more: the fold goes back to in place (the global state keeps its packed storage)
    del v, held
    m._computed = None
    ptr = m.a.untyped_storage().data_ptr()
    m(torch.ones(4))
    assert m.a.untyped_storage().data_ptr() == ptr and m.a.tolist() == [4.0] * 4


@pytest.mark.parametrize("hand_out", ["attr", "compute_same_object", "state_dict", "metric_state", "view",
                                      "collection_sibling"])
def test_reset_never_zeroes_a_handed_out_state(hand_out):
    """reset() refills a state in place only when nothing outside the metric can observe it; every path that hands a
    state (or a view of it) out must keep its value across reset()."""
    p, t = _data(3)
    if hand_out == "collection_sibling":
        coll = MetricCollection([tm.MulticlassPrecision(5, average=None), tm.MulticlassRecall(5, average=None)],
                                compute_groups=True)
        coll.update(p, t)
        coll.compute()
        m = coll["MulticlassPrecision"]
        held = coll["MulticlassRecall"].tp
    else:
        m = _ViewCompute() if hand_out == "compute_same_object" else tm.MulticlassStatScores(5, average=None)
        if hand_out == "compute_same_object":
            m.compute = lambda: m.a  # returns the state object itself
            m.update(torch.ones(4))
            held = m.a
        else:
            m.persistent(True)
            m.update(p, t)
            held = {"attr": lambda: m.tp, "state_dict": lambda: m.state_dict(keep_vars=True)["tp"],
                    "metric_state": lambda: m.metric_state["tp"], "view": lambda: m.tp[1:]}[hand_out]()
    before = held.clone()
    m.reset()
    assert torch.equal(held, before)


@pytest.mark.parametrize("hand_out", ["attr", "metric_state", "state_dict", "in_list", "in_dict", "compute_result"])
def test_forward_never_mutates_a_handed_out_state_object(hand_out):
    """forward()'s in-place fold must not change a state OBJECT (not a view) the user holds through any hand-out path,
    including containers; the guard is the exact strong-reference count read from C (ops.sole_ref), not
    sys.getrefcount's version-dependent conventions."""
    p, t = _data(3)
    m = tm.MulticlassConfusionMatrix(5) if hand_out == "compute_result" else tm.MulticlassStatScores(5, average=None)
    m.persistent(True)
    m.update(p, t)
    key = "confmat" if hand_out == "compute_result" else "tp"
    get = {"attr": lambda: getattr(m, key), "metric_state": lambda: m.metric_state[key],
           "state_dict": lambda: m.state_dict(keep_vars=True)[key], "in_list": lambda: [getattr(m, key)],
           "in_dict": lambda: {"x": getattr(m, key)}, "compute_result": lambda: m.compute()}[hand_out]
    held = get()
    obj = held[0] if hand_out == "in_list" else held["x"] if hand_out == "in_dict" else held
    before = obj.clone()
    del obj
    m(p, t)
    obj = held[0] if hand_out == "in_list" else held["x"] if hand_out == "in_dict" else held
    assert torch.equal(obj, before)
    m.reset()
    assert torch.equal(obj, before)


def test_sole_ref_probe_counts_every_holder():
    from torchmetrics_amd import ops

    if not ops.native_available():
        pytest.skip("native library not built")
    d = {"x": torch.zeros(3)}
    assert ops.sole_ref(d, "x")
    held = [d["x"]]
    assert not ops.sole_ref(d, "x")
    held.clear()
    assert ops.sole_ref(d, "x")
    y = d["x"]
    assert not ops.sole_ref(d, "x")
    del y
    assert ops.sole_ref(d, "x") and not ops.sole_ref(d, "missing") and not ops.sole_ref({"a": 1}, "a")
