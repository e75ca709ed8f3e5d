"""ORACLE — test infrastructure only.

A CPU restatement of the reference's hot path (NEPTUNE's placement MIP as handed to
OR-Tools/SCIP) used as the *checker* of the MI355X implementation:

  oracle.inputs       restates `core/utils/input_to_data.py:88-286` (payload -> matrices)
  oracle.formulation  restates the model builders `core/solvers/neptune/utils/*.py` and the
                      step classes `neptune_step1.py` / `neptune_step2.py` as one CSR model
                      (same variable order, same row order, same coefficients)
  oracle.solve        HiGHS (scipy) on that CSR: LP relaxations, MIPs, and the two-step flow of
                      `core/solvers/neptune/neptune.py:18-39` plus the output wire format of
                      `neptune/utils/output.py:23-39`

Pinning: the restated CSR is compared entry-by-entry against the models the reference's own
builders recorded (tests/golden/models/*.npz, produced by tools/gen_golden.py), and the flow's
responses against the reference's committed SCIP outputs (`output-mip.json`, Alibaba
`testing/alibaba/alibaba_test/output_*_case0.json`).  The real engine (OR-Tools 9.6.2534 +
SCIP, `requirements.txt:8`) is not installable offline; HiGHS stands in for it.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
The product path (neptune-mip_amd/) never does.
"""
