"""pyorbslam_amd — MI355X-native (gfx950 HIP) ORB front-end for pyOrbSLAM2.

Hot path (BASELINE.json north_star): ORB extraction of the left and right images (FAST pyramid,
octree distribution, IC angle, 256-bit steered BRIEF), Frame.compute_stereo_matches and the ORBMatcher
Hamming search, all in hand-written HIP kernels behind the C-ABI of include/orbfe.h (liborbfe.so).

  pyorbslam_amd.pyORBExtractor.ORBextractor   drop-in for the reference pybind11 class
  pyorbslam_amd.frame.compute_stereo_matches  drop-in for Frame.compute_stereo_matches
  pyorbslam_amd.matcher.ORBMatcher            drop-in for ORBMatcher's projection searches
  pyorbslam_amd.batch.StereoFrontEnd          batched device-resident stereo pairs (throughput path)
  pyorbslam_amd.dist                          one process per GPU, pairs sharded across ranks
"""
__version__ = "0.1.0"
