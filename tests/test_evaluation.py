"""RecommenderEvaluator (src/evaluation.py:19-149) against goldens produced by
executing the reference (tests/golden/evaluation.json, make_golden.py).

CPU: NDCG, MAE/RMSE and _binarize (host arithmetic through the same sklearn
calls). GPU: Precision@k / Recall@k, whose ranking step is the device's stable
top-k, and comprehensive_evaluation (raises ValueError like the reference, D7).
Exact equality.
"""
import pytest

from conftest import load_golden


def _cases():
    return load_golden("evaluation.json")["cases"]


def _dict(pairs):
    return {int(i): v for i, v in pairs}


def _check(got_fn, exp):
    if "raises" in exp:
        with pytest.raises(Exception) as ei:
            got_fn()
        assert type(ei.value).__name__ == exp["raises"]
    else:
        assert got_fn() == exp["ok"]


def _evaluator():
    from src.evaluation import RecommenderEvaluator

    return RecommenderEvaluator()


def test_ndcg_mae_binarize_comprehensive_match_reference():
    ev = _evaluator()
    for c in _cases():
        a, p = _dict(c["actual"]), _dict(c["pred"])
        for k, exp in c["ndcg"]:
            _check(lambda: float(ev.ndcg_at_k(a, p, k)), exp)
        _check(lambda: [float(x) for x in ev.mae_rmse(a, p)], c["mae_rmse"])
        assert [[i, v] for i, v in ev._binarize(a).items()] == c["binarize"]


@pytest.mark.gpu
def test_precision_recall_at_k_match_reference():
    ev = _evaluator()
    for c in _cases():
        a, p = _dict(c["actual"]), _dict(c["pred"])
        for k, exp in c["precision"]:
            _check(lambda: ev.precision_at_k(a, p, k), exp)
        for k, exp in c["recall"]:
            _check(lambda: ev.recall_at_k(a, p, k), exp)
        _check(lambda: ev.comprehensive_evaluation(a, p), c["comprehensive"])  # D7: ValueError


@pytest.mark.gpu
def test_ranked_items_negative_and_large_k():
    from src.evaluation import ranked_items

    p = {5: 1.0, 3: 2.0, 9: 2.0, 1: -1.0}
    assert ranked_items(p, 10) == [3, 9, 5, 1]
    assert ranked_items(p, -1) == [3, 9, 5]
    assert ranked_items(p, 0) == []
