"""CPU ORACLE — test infrastructure only, never the product path.

A plain PyTorch-CPU fp32 restatement of the reference's hot path
(RUA1027/Lowlight_Image_Enhancement): NAFNet forward/backward (Scenario B), the
crosstalk-PSF physics branch and the HybridLoss terms.  Every function cites the
reference file:line it restates.

Who may import this package: `tests/`, `__graft_entry__.smoke()` (as the checker)
and `bench.py`'s `cpu_baseline` leg.  The MI355X product
(`lowlight_image_enhancement_amd/`) never imports it and has no CPU fallback.

Pinning: every restated function is checked against fixtures that were produced
by running the reference itself (tests/golden/make_golden.py, stub-import recipe
of SURVEY.md §8c) — see tests/test_oracle_golden.py.  Exceptions, documented as
"parity unpinned" in DESIGN.md: the kornia-0.6.12 SSIMLoss and rgb_to_lab
restatements (kornia is not installed here; SSIM is partially pinned through the
reference's own metrics/linear.ssim_linear, see tests).
"""
