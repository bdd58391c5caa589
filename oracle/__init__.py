"""CPU oracle for the frame-synthesis hot path — TEST INFRASTRUCTURE ONLY.

A plain PyTorch-CPU fp32 restatement of the reference's algorithm (HRNet coarse
generator, RGBLoss components, cross-entropy, PSNR, flow warp, one InterTrainer step with
Adamax), written from the reference sources' behaviour; each function cites the
reference file:line it follows.  Pinned against golden vectors generated from the
reference itself (tests/golden/make_golden.py imports /root/reference with offline stubs
and records its outputs; tests/test_oracle_golden.py checks this package against them).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / CPU baseline.  The product path (the package
deep_video_interpolation_extrapolation_amd) never imports it and has no CPU fallback.
"""
