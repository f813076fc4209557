"""Joint trees of the dataset skeletons (drop-in for the reference's common/skeleton.py).

Same class and methods as the reference's `Skeleton` (skeleton.py:10-88):
num_joints, parents, has_children, children, remove_joints, joints_left,
joints_right.  `remove_joints` re-parents every kept joint to its nearest kept
ancestor, renumbers the kept joints densely in their original order and drops the
removed ones from the left/right symmetry lists; it returns the kept joint indices
(the column selection the datasets apply to their positions).
"""
import numpy as np


class Skeleton:
    def __init__(self, parents, joints_left, joints_right):
        assert len(joints_left) == len(joints_right)
        self._parents = np.array(parents)
        self._joints_left = list(joints_left) if joints_left is not None else None
        self._joints_right = list(joints_right) if joints_right is not None else None
        self._compute_metadata()

    def num_joints(self):
        return len(self._parents)

    def parents(self):
        return self._parents

    def has_children(self):
        return self._has_children

    def children(self):
        return self._children

    def joints_left(self):
        return self._joints_left

    def joints_right(self):
        return self._joints_right

    def remove_joints(self, joints_to_remove):
        drop = set(int(j) for j in joints_to_remove)
        n = len(self._parents)
        kept = [j for j in range(n) if j not in drop]
        parents = [int(p) for p in self._parents]
        for i in range(n):  # climb to the nearest kept ancestor
            while parents[i] in drop:
                parents[i] = parents[parents[i]]
        new_index = {j: k for k, j in enumerate(kept)}
        self._parents = np.array([new_index[parents[j]] if parents[j] >= 0 else -1 for j in kept])
        if self._joints_left is not None:
            self._joints_left = [new_index[j] for j in self._joints_left if j in new_index]
        if self._joints_right is not None:
            self._joints_right = [new_index[j] for j in self._joints_right if j in new_index]
        self._compute_metadata()
        return kept

    def _compute_metadata(self):
        n = len(self._parents)
        self._has_children = np.zeros(n, dtype=bool)
        self._children = [[] for _ in range(n)]
        for i, p in enumerate(self._parents):
            if p != -1:
                self._has_children[p] = True
                self._children[p].append(i)
