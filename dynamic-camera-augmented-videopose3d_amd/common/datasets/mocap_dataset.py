"""Base dataset (drop-in for the reference's common/datasets/mocap_dataset.py:11-48).

Differences: `remove_joints` works on the 2D and 3D skeletons the base class actually
keeps (the reference calls `self._skeleton`, which no class sets: quirk Q1, the
AttributeError that stops Human36mDataset(remove_static_joints=True)); each
skeleton object is edited once even when 2D and 3D share it; positions of every
sequence keep the kept joints only.
"""


class MocapDataset:
    def __init__(self, fps, skeleton_2d, skeleton_3d):
        self._skeleton_2d = skeleton_2d
        self._skeleton_3d = skeleton_3d
        self._fps = fps
        self._data = None  # filled by the subclass
        self._cameras = None

    def remove_joints(self, joints_to_remove):
        kept = None
        seen = []
        for sk in (self._skeleton_3d, self._skeleton_2d):
            if any(sk is s for s in seen):
                continue
            seen.append(sk)
            k = sk.remove_joints(joints_to_remove)
            kept = k if kept is None else kept
        for subject in self._data.values():
            for s in subject.values():
                if "positions" in s:
                    s["positions"] = s["positions"][:, kept]
        return kept

    def __getitem__(self, key):
        return self._data[key]

    def subjects(self):
        return self._data.keys()

    def fps(self):
        return self._fps

    def skeleton_2d(self):
        return self._skeleton_2d

    def skeleton_3d(self):
        return self._skeleton_3d

    def cameras(self):
        return self._cameras

    def supports_semi_supervised(self):
        return False
