"""CPU oracle for the NRMS scoring path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package. The product path
(``newsrecommendationsystem_amd``) never imports it and has no CPU fallback.

Contents:
  weights.py        deterministic, numpy-version-independent parameter/input
                    generator (splitmix64) shared by the golden script, the
                    tests and the bench.
  nrms_oracle.py    numpy restatement of the reference NRMS forward path
                    (src/model/NRMS/*, src/model/general/*), fp32 or fp64.
  nrms_torch_cpu.py the same algorithm as the reference's ATen op sequence on
                    CPU tensors: the timed CPU baseline (kind "port").
  metrics.py        restatement of the evaluation metrics (src/evaluate.py).

Parity is pinned: tests/golden/nrms_golden.npz was produced by importing the
reference model in the build container (tests/golden/gen_golden.py), and
tests/test_oracle_golden.py checks both restatements against it.
"""
