"""Generate golden vectors by EXECUTING the reference's own Python functions.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):   python tests/golden/make_golden.py

The reference package cannot be imported as-is: its engines (pyspark,
tensorflow) and plotting deps (matplotlib, seaborn) are not installed, and two
of its own imports are broken (D1: src/als_model.py:17 imports a
get_item_features that src/data_preprocessing.py never defines; D2:
src/hybrid_system.py:15 imports compute_f1_score from evaluation, which lives
in als_model). This script therefore registers empty stand-in modules for the
missing third-party packages (only their names are looked up at import time;
no function exercised below calls into them), loads the reference modules
from their files without running src/__init__.py, and patches D1/D2 with
placeholders. Every number written below comes from the reference's code:

  * HybridRecommendationSystem.adaptive_fusion / get_hybrid_recommendations
    (src/hybrid_system.py:57-75, 95-116) with duck-typed model objects;
  * compute_f1_score (src/als_model.py:171-177, src/two_tower_model.py:238-245);
  * ALSModel._find_similar_items (src/als_model.py:93-104) and the fallback
    loop of ALSModel.predict_for_user (:68-91) with a fake Spark model that
    returns fixed predictions;
  * TwoTowerModel.predict_for_user input assembly (src/two_tower_model.py:136-146)
    and _prepare_features (:123-134) with a recording fake Keras model;
  * utils.scale_ratings_to_5 / normalize_predictions (src/utils.py:16-79);
  * RecommenderEvaluator precision/recall/NDCG/MAE-RMSE/_binarize and the
    comprehensive_evaluation entry point (src/evaluation.py:19-149).

Output: tests/golden/*.json (data only: inputs and expected outputs).
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np
import pandas as pd
import sklearn

REF = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------- harness
def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    sys.modules[name] = mod
    return mod


class _Opaque:
    def __init__(self, *a, **k):
        raise RuntimeError("engine stand-in: not available in this container")


def install_stubs():
    _stub("pyspark")
    _stub("pyspark.sql", SparkSession=_Opaque)
    _stub("pyspark.sql.types", StructType=lambda *a, **k: None, StructField=lambda *a, **k: None,
          IntegerType=lambda *a, **k: None)
    _stub("pyspark.ml")
    _stub("pyspark.ml.recommendation", ALS=_Opaque, ALSModel=_Opaque)
    _stub("tensorflow")
    _stub("tensorflow.keras")
    _stub("tensorflow.keras.models", Model=_Opaque, save_model=_Opaque)
    _stub("tensorflow.keras.layers", Input=_Opaque, Embedding=_Opaque, Flatten=_Opaque,
          Dense=_Opaque, Concatenate=_Opaque, Dot=_Opaque, LayerNormalization=_Opaque)
    _stub("tensorflow.keras.optimizers", Adam=_Opaque)
    _stub("tensorflow.keras.callbacks", EarlyStopping=_Opaque, ModelCheckpoint=_Opaque)
    _stub("seaborn")
    _stub("matplotlib")
    _stub("matplotlib.pyplot")


def load_reference():
    install_stubs()
    pkg = types.ModuleType("refsrc")
    pkg.__path__ = [REF]
    sys.modules["refsrc"] = pkg

    def load(name):
        spec = importlib.util.spec_from_file_location(f"refsrc.{name}", os.path.join(REF, f"{name}.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[f"refsrc.{name}"] = mod
        spec.loader.exec_module(mod)
        return mod

    dp = load("data_preprocessing")
    dp.get_item_features = lambda data: None  # D1 placeholder (never called here)
    als = load("als_model")
    ev = load("evaluation")
    ev.compute_f1_score = als.compute_f1_score  # D2
    tt = load("two_tower_model")
    hy = load("hybrid_system")
    ut = load("utils")
    return types.SimpleNamespace(als=als, tt=tt, hy=hy, ut=ut, ev=ev)


# ------------------------------------------------------------- encoding
def enc_score(x):
    """JSON-safe scalar with its numpy dtype (exact round trip)."""
    if isinstance(x, np.floating):
        return {"v": float(x), "t": str(x.dtype)}
    if isinstance(x, (int, np.integer)) and not isinstance(x, bool):
        return {"v": int(x), "t": "int"}
    return {"v": float(x), "t": "float"}


def enc_pairs(pairs):
    return [[int(i), enc_score(s)] for i, s in pairs]


class FakeModel:
    def __init__(self, preds):
        self.preds = preds

    def predict_for_user(self, user_id, all_items):
        return list(self.preds)


# ---------------------------------------------------------------- cases
def fusion_cases(ref, rng):
    cases = []

    def add(name, als_preds, tt_preds, als_f1, tt_f1, top_k):
        hrs = ref.hy.HybridRecommendationSystem()
        hrs.als_f1_score, hrs.twotower_f1_score = als_f1, tt_f1
        combined = hrs.adaptive_fusion(als_preds, tt_preds)
        hrs2 = ref.hy.HybridRecommendationSystem()
        hrs2.models_loaded = True
        hrs2.als_f1_score, hrs2.twotower_f1_score = als_f1, tt_f1
        hrs2.als_model, hrs2.twotower_model = FakeModel(als_preds), FakeModel(tt_preds)
        top = hrs2.get_hybrid_recommendations(0, [], top_k=top_k)
        cases.append({
            "name": name, "als_f1": als_f1, "tt_f1": tt_f1, "top_k": top_k,
            "als": enc_pairs(als_preds), "tt": enc_pairs(tt_preds),
            "combined": enc_pairs(combined), "top": enc_pairs(top),
        })

    n = 20
    ids = list(range(n))
    add("dense_f64", [(i, float(rng.normal())) for i in ids], [(i, float(rng.normal())) for i in ids],
        0.0, 0.0, 5)
    add("dense_tt_f32", [(i, float(rng.normal() * 3)) for i in ids],
        [(i, np.float32(rng.normal())) for i in ids], 0.3, 0.1, 5)
    add("tt_missing_items", [(i, float(rng.uniform(0, 18))) for i in ids],
        [(i, np.float32(rng.normal())) for i in ids[:12]], 0.1, 0.4, 10)
    add("als_missing_items", [(i, float(rng.uniform(0, 18))) for i in ids[5:]],
        [(i, float(rng.normal())) for i in ids], 0.5, 0.5, 5)
    q = [(i, float(np.round(rng.uniform(0, 4)))) for i in ids]
    add("ties_quantised", q, [(i, float(np.round(rng.uniform(0, 2)))) for i in ids], 0.0, 0.0, 10)
    add("constant_both", [(i, 3.0) for i in ids], [(i, np.float32(0.25)) for i in ids], 0.2, 0.1, 5)
    add("constant_als", [(i, 2.5) for i in ids], [(i, float(rng.normal())) for i in ids], 0.0, 0.2, 5)
    big = list(range(0, 600, 3))
    add("n200_quantised_f32", [(i, float(np.round(rng.normal(), 1))) for i in big],
        [(i, np.float32(np.round(rng.normal(), 2))) for i in big], 0.0, 0.0, 10)
    sparse_ids = [int(x) for x in rng.choice(10 ** 9, size=30, replace=False)]
    add("sparse_ids", [(i, float(rng.normal())) for i in sparse_ids],
        [(i, float(rng.normal())) for i in sparse_ids], 0.9, 0.1, 5)
    add("empty_tt", [(i, float(rng.normal())) for i in ids], [], 0.0, 0.0, 5)
    add("top_k_exceeds_n", [(i, float(rng.normal())) for i in ids[:3]],
        [(i, float(rng.normal())) for i in ids[:3]], 0.0, 0.0, 10)
    return cases


def f1_cases(ref, rng):
    out = []
    for t in range(12):
        n_act = int(rng.integers(0, 6))
        n_pred = int(rng.integers(0, 25))
        actual = {int(i): float(rng.uniform(0, 5)) for i in rng.choice(30, n_act, replace=False)}
        pred = {int(i): float(np.round(rng.normal(), 1)) for i in rng.choice(30, n_pred, replace=False)}
        for k in (10, 5, 0):
            rec = {"actual": [[i, s] for i, s in actual.items()], "pred": [[i, s] for i, s in pred.items()],
                   "k": k}
            for name, fn in (("als", ref.als.compute_f1_score), ("tt", ref.tt.compute_f1_score)):
                try:
                    rec[name] = float(fn(actual, pred, k=k))
                except ZeroDivisionError:
                    rec[name] = "ZeroDivisionError"
            out.append(rec)
    return out


def similar_cases(ref, rng):
    out = []
    for t in range(4):
        n_items = 40
        feats = {}
        prev = None
        for i in range(n_items):
            f = rng.normal(size=3)
            if i % 7 == 3 and prev is not None:
                f = prev.copy()  # exact duplicate of the previous item -> ties
            if i == 11:
                f = np.zeros(3)
            prev = f
            feats[i * 2 + t] = {"features": np.asarray(f, dtype=np.float64),
                                "rating": float(rng.integers(0, 19))}
        m = ref.als.ALSModel()
        m.item_features = feats
        queries = list(feats.keys())[:12] + [10 ** 6]
        res = {str(q): [int(x) for x in m._find_similar_items(q)] for q in queries}
        out.append({
            "item_features": [[int(i), [float(x) for x in d["features"]], d["rating"]] for i, d in feats.items()],
            "queries": [int(q) for q in queries],
            "similar": res,
        })
    return out


class _Row:
    def __init__(self, itemId, prediction):
        self.itemId, self.prediction = itemId, prediction


class _FakeDF:
    def __init__(self, rows):
        self.rows = rows

    def collect(self):
        return self.rows


def als_fallback_cases(ref, rng):
    """ALSModel.predict_for_user with a fake Spark model: pins the fallback."""
    out = []
    for t in range(3):
        n_items = 25
        item_ids = [int(i) for i in rng.choice(1000, n_items, replace=False)]
        feats = {i: {"features": rng.normal(size=3), "rating": float(rng.integers(0, 19))} for i in item_ids}
        known = {i: float(np.float32(rng.normal() * 4)) for i in item_ids if rng.uniform() < 0.6}
        nan_items = [i for i in known if rng.uniform() < 0.15]
        spark_rows = [_Row(i, float("nan") if i in nan_items else v) for i, v in known.items()]
        query = item_ids + [5000 + t]  # one id without features -> global_mean

        class FakeSpark:
            def createDataFrame(self, pairs, schema=None):
                return pairs

        class FakeSparkModel:
            def transform(self, df):
                return _FakeDF(spark_rows)

        m = ref.als.ALSModel()
        m.spark, m.model = FakeSpark(), FakeSparkModel()
        m.item_features = feats
        m.global_mean = float(rng.uniform(0, 18))
        res = m.predict_for_user(7, query)
        out.append({
            "item_features": [[i, [float(x) for x in feats[i]["features"]], feats[i]["rating"]] for i in item_ids],
            "spark_predictions": [[r.itemId, r.prediction if r.prediction == r.prediction else None]
                                  for r in spark_rows],
            "global_mean": m.global_mean, "query": query,
            "result": enc_pairs(res),
        })
    return out


def tt_input_cases(ref, rng):
    from sklearn.preprocessing import MinMaxScaler

    out = []
    for t in range(2):
        n = 15
        train = pd.DataFrame({
            "userId": rng.integers(0, 50, n), "itemId": rng.integers(0, 80, n),
            "manufacturer_id": rng.integers(0, 9, n), "category_id": rng.integers(0, 4, n),
            "price": np.round(rng.uniform(1, 300, n), 2), "average_review_rating": rng.integers(0, 19, n),
        })
        m = ref.tt.TwoTowerModel(50, 80, 9, 4)
        feats = m._prepare_features(train)  # fits the scaler (D10)
        cand = pd.DataFrame({
            "itemId": rng.integers(0, 80, 9), "manufacturer_id": rng.integers(0, 9, 9),
            "category_id": rng.integers(0, 4, 9), "price": np.round(rng.uniform(0, 400, 9), 2),
            "average_review_rating": rng.integers(0, 19, 9),
        })
        rec = {}

        class Recorder:
            def predict(self, inputs, verbose=0):
                rec.update(inputs)
                return (np.arange(len(inputs["user_in"]), dtype=np.float32) * np.float32(0.5)).reshape(-1, 1)

        m.model = Recorder()
        res = m.predict_for_user(31, cand)
        out.append({
            "train": train.to_dict(orient="list"), "candidates": cand.to_dict(orient="list"),
            "prepare_numeric_in": feats["numeric_in"].tolist(),
            "scaler_min": m.scaler.data_min_.tolist(), "scaler_max": m.scaler.data_max_.tolist(),
            "inputs": {k: np.asarray(v).tolist() for k, v in rec.items()},
            "input_dtypes": {k: str(np.asarray(v).dtype) for k, v in rec.items()},
            "result": enc_pairs(res),
        })
    return out


def utils_cases(ref):
    return {
        "scale_ratings_to_5": [[[1, 2, 3, 4, 5], ref.ut.scale_ratings_to_5([1, 2, 3, 4, 5])],
                               [[2.0, 2.0], ref.ut.scale_ratings_to_5([2.0, 2.0])],
                               [[0, 18, 9], ref.ut.scale_ratings_to_5([0, 18, 9])]],
        "normalize_predictions": [[[[i, s] for i, s in {1: 0.5, 2: 3.0, 7: -1.0}.items()],
                                   [[int(i), float(s)] for i, s in
                                    ref.ut.normalize_predictions({1: 0.5, 2: 3.0, 7: -1.0}).items()]]],
    }


def _exc(fn):
    """Value of fn(), or the name of the exception it raises."""
    try:
        return {"ok": fn()}
    except Exception as e:  # noqa: BLE001 - the exception type is the expected output
        return {"raises": type(e).__name__}


def evaluation_cases(ref):
    """RecommenderEvaluator (src/evaluation.py:19-149) on per-user dicts.
    Dicts are stored as [key, value] lists in insertion order."""
    rng = np.random.default_rng(7)
    ev = ref.ev.RecommenderEvaluator()
    cases = []
    for c in range(40):
        n_act = int(rng.integers(1, 40))
        items = rng.choice(200, size=n_act + 30, replace=False).tolist()
        if c % 3 == 0:
            actual = {int(i): int(rng.integers(0, 19)) for i in items[:n_act]}
        else:
            actual = {int(i): float(np.round(rng.uniform(1, 5), 1)) for i in items[:n_act]}
        pred_items = items[n_act // 2: n_act // 2 + int(rng.integers(1, 45))]
        if c % 4 == 1:
            pred = {int(i): float(np.round(rng.uniform(0, 5), 0)) for i in pred_items}  # many ties
        elif c % 4 == 2:
            pred = {int(i): float(rng.normal()) for i in pred_items}
        else:
            pred = {int(i): float(np.float32(rng.uniform(1, 5))) for i in pred_items}
        if c == 5:
            pred = {i: 3.0 for i in pred}  # all tied
        if c == 6:
            actual = {i: 4 for i in actual}  # constant truth
        k_vals = [0, 1, 3, 5, 10, 15, 20] if c % 5 == 0 else [5, 10]
        case = {"actual": [[i, v] for i, v in actual.items()], "pred": [[i, v] for i, v in pred.items()],
                "precision": [[k, _exc(lambda k=k: ev.precision_at_k(actual, pred, k))] for k in k_vals if k > 0],
                "recall": [[k, _exc(lambda k=k: ev.recall_at_k(actual, pred, k))] for k in k_vals],
                "ndcg": [[k, _exc(lambda k=k: float(ev.ndcg_at_k(actual, pred, k)))] for k in (5, 10)],
                "mae_rmse": _exc(lambda: [float(x) for x in ev.mae_rmse(actual, pred)]),
                "binarize": [[i, v] for i, v in ev._binarize(actual).items()],
                "comprehensive": _exc(lambda: {kk: float(vv) for kk, vv in
                                               ev.comprehensive_evaluation(actual, pred).items()})}
        cases.append(case)
    return cases


def main():
    ref = load_reference()
    rng = np.random.default_rng(20250620)
    meta = {"numpy": np.__version__, "sklearn": sklearn.__version__, "python": sys.version.split()[0],
            "generator": "tests/golden/make_golden.py"}
    files = {
        "fusion.json": fusion_cases(ref, rng),
        "f1.json": f1_cases(ref, rng),
        "similar_items.json": similar_cases(ref, rng),
        "als_fallback.json": als_fallback_cases(ref, rng),
        "tt_inputs.json": tt_input_cases(ref, rng),
        "utils.json": utils_cases(ref),
        "evaluation.json": evaluation_cases(ref),
    }
    for name, data in files.items():
        with open(os.path.join(OUT, name), "w") as f:
            json.dump({"meta": meta, "cases": data}, f, indent=1, default=lambda o: o.item())
        print("wrote", name)


if __name__ == "__main__":
    main()
