"""CPU oracle for the hybrid ALS + two-tower hot path — TEST INFRASTRUCTURE.

This package restates, on the CPU, the arithmetic the reference delegates to
its engines (Spark 3.5.1 explicit ALS, Keras 2.8 two-tower, sklearn
MinMaxScaler + Python's stable sort in the fusion). It is the checker for the
HIP path, never the product: only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import it. The shipped package
(hybrid-als-twotower-recommender_amd/src) must not import anything from here.

Parity status (details: DESIGN.md §Oracle):
  * fusion / top-k / F1 / similar-items / TT input assembly: pinned against
    golden vectors produced by executing the reference's own Python functions
    (tests/golden/make_golden.py);
  * ALS: restated from Spark 3.5.1 ALS.scala [ext, not in /root/reference];
    the solve calls the very LAPACK routine Spark calls (dppsv, via scipy) on
    Spark's packed-upper layout; pinned by analytic known answers. Spark
    itself is not installed -> the Spark-engine result is "parity unpinned"
    beyond that.
  * two-tower: restated from Keras 2.8 layers/Adam [ext]; TF is not
    installed -> "parity unpinned" beyond closed-form checks.
"""
