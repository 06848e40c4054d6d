"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

A plain torch-CPU / numpy restatement of RVC-MAKER's voice-conversion hot path
(``main/inference/convert.py:VC.pipeline``), written from SURVEY.md §8 and the
reference sources, never copied from them.  Every function cites the reference
file:line it follows.

Rules (DESIGN.md "Oracle"):
* Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import this package, and only as the checker or the
  timed CPU baseline.  The product path (``rvc-maker_amd/rvc_amd``) never
  imports it and fails loudly when its HIP library is missing.
* Parity pinning: the restatement is checked against golden vectors produced by
  running the reference itself in the survey container
  (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``).  Pieces the
  reference could not run here are marked "parity unpinned" where they appear
  (librosa mel basis; FAISS).
"""
