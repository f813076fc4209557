"""MI355X-native drop-in for the reference's ``common`` package (hot-path modules only).

Put ``dynamic-camera-augmented-videopose3d_amd/`` ahead of the reference on
PYTHONPATH and ``from common.models.TemporalModel import *`` resolves here.
"""
