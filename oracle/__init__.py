"""CPU oracle for the hetero-SAGE hot path — TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg,
as the checker.  Never imported by ``truth_recommendation_gnn_amd``.  Parity status: see the
header of ``oracle/sage_ref.py`` ("parity unpinned" against the reference; pinned by the float64
dense formulation in ``oracle/dense_ref.py``).
"""
