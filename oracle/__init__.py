"""CPU oracle for the Dreamer world-model / imagination hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and only
as the checker (or the timed CPU baseline). The product path (safe-dreamer_amd/sdreamer) never imports it.

Contents:
  noise.py  — Philox4x32-10 counter-based noise (gumbel / normal) shared by oracle and HIP kernels.
  init.py   — deterministic parameter generator used to give reference, oracle and product identical weights.
  ref_cpu.py— fp32 PyTorch-CPU restatement of the reference path, op for op, citing reference file:line.
Parity pin: tests/golden/*.npz were produced by importing the real reference in the survey container
(tests/golden/gen_golden.py); tests/test_oracle_golden.py checks this restatement against them.
"""
