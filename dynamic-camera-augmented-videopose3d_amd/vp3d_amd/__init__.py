"""vp3d_amd — MI355X-native VideoPose3D temporal lifter (host side of libvp3d.so).

Modules
  _native   ctypes binding of include/vp3d.h (no fallback)
  lifter    NativeLifter: one vp3d_handle (folded weights + workspace) per device
  pipeline  on-device input path: normalisation, K·E, window gather, mpjpe
  synth     seeded counter-hash synthetic weights / keypoints / cameras
  shard     embarrassingly parallel batch sharding over ranks (no collective)
  build     in-tree hipcc build of libvp3d.so for gfx950
"""
__version__ = "0.1.0"
