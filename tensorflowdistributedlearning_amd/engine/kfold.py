"""Stratified K-fold splitting (the reference uses sklearn's ``StratifiedKFold(n_splits, shuffle=True,
random_state=seed)``, model.py:134-136,149-154).

Own implementation (no sklearn dependency in the training path) of the same algorithm: per class,
shuffled indices are dealt round-robin-balanced into folds so every fold keeps the class
proportions (classes numbered by first appearance, fold ids shuffled per class with
``RandomState(seed)``).  tests/test_engine_cpu.py checks index-for-index equality with sklearn.
"""
from __future__ import annotations

import numpy as np


class StratifiedKFold:
    def __init__(self, n_splits=5, shuffle=True, random_state=None):
        if n_splits < 2:
            raise ValueError("n_splits must be >= 2")
        self.n_splits = n_splits
        self.shuffle = shuffle
        self.random_state = random_state

    def _test_folds(self, y):
        y = np.asarray(y)
        _, first_idx, y_inv = np.unique(y, return_index=True, return_inverse=True)
        # classes numbered by order of first appearance (sklearn's encoding)
        _, class_perm = np.unique(first_idx, return_inverse=True)
        y_enc = class_perm[y_inv.reshape(-1)]
        n_classes = len(first_idx)
        counts = np.bincount(y_enc)
        if np.all(self.n_splits > counts):
            raise ValueError("n_splits cannot be greater than the number of members in each class")
        # sklearn: sort by class, then allocate fold ids so each fold gets ~count/n_splits per class
        y_order = np.sort(y_enc)
        allocation = np.asarray([np.bincount(y_order[i::self.n_splits], minlength=n_classes)
                                 for i in range(self.n_splits)])
        rng = np.random.RandomState(self.random_state) if self.shuffle else None
        test_folds = np.empty(len(y), dtype=np.int64)
        for k in range(n_classes):
            folds_for_class = np.arange(self.n_splits).repeat(allocation[:, k])
            if rng is not None:
                rng.shuffle(folds_for_class)
            test_folds[y_enc == k] = folds_for_class
        return test_folds

    def split(self, X, y):
        n = len(X)
        y = np.asarray(y)
        if len(y) != n:
            raise ValueError("X and y have different lengths")
        folds = self._test_folds(y)
        idx = np.arange(n)
        for f in range(self.n_splits):
            test = idx[folds == f]
            train = idx[folds != f]
            yield train, test

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.n_splits
