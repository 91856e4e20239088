"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the articulated-point render/deform path.

This package is the *checker*: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The product path
(``articulated-point-nerf_amd/apn_amd``) never imports, links or executes anything here
and fails loudly when its HIP library is missing.

Pinning: ``tests/golden/make_golden.py`` runs the reference's own Python
(``lib/temporalpoints.py``, ``lib/pointwarper.py``, ``lib/tineuvox.py``, imported with
stubbed third-party modules) on synthetic inputs and stores the outputs under
``tests/golden/``; ``tests/test_oracle_golden.py`` checks this oracle against them.
The reference CUDA kernels (render_utils_kernel.cu) cannot be built here,
so their restatement below is pinned by the kernel source text and by hand-derived
known-answer tests (``tests/test_oracle_kernels.py``).
"""
