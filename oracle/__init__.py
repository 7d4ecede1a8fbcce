"""TEST INFRASTRUCTURE ONLY — CPU checkers for the gfx950 front-end.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.  The
product (pyorbslam_amd) never imports it and fails loudly when its HIP library is missing.

  orb_oracle.cpp / oracle.py   C++ restatement of pyORBExtractor/ORBextractor.cpp + the OpenCV 4.x
                               primitives it calls.  Parity UNPINNED (OpenCV absent; no reference
                               extractor fixtures exist).
  stereo_oracle.py             numpy restatement of Frame.compute_stereo_matches (Frame.py:161-279).
                               Pinned against tests/golden/stereo_*.npz produced by the imported
                               reference method.
  matcher_oracle.py            restatement of ORBMatcher's Hamming searches (ORBMatcher.py:12-14,
                               215-283, 291-393), pinned against tests/golden/matcher_*.json.
"""
