"""Trainset, mirroring surprise/trainset.py:11-261, stored array-natively.

The reference keeps ``ur`` / ``ir`` as dict-of-lists and walks them with the
``all_ratings()`` generator (trainset.py:180-190).  Here the canonical storage
is a user-major CSR in exactly that iteration order (users by inner id, each
user's ratings in insertion order), which is what the HIP kernels consume;
``ur`` / ``ir`` are materialised lazily for API compatibility only.
"""
from collections import defaultdict

import numpy as np


class _IdentityIds:
    """raw id -> inner id map for array-native datasets whose raw ids are 0..n-1."""

    def __init__(self, n):
        self.n = int(n)

    def __getitem__(self, key):
        if isinstance(key, (int, np.integer)) and 0 <= int(key) < self.n:
            return int(key)
        raise KeyError(key)

    def __contains__(self, key):
        return isinstance(key, (int, np.integer)) and 0 <= int(key) < self.n

    def items(self):
        return ((k, k) for k in range(self.n))

    def __len__(self):
        return self.n


class Trainset:
    """See surprise/trainset.py:11-60 for the attribute contract."""

    def __init__(self, ur, ir, n_users, n_items, n_ratings, rating_scale, offset,
                 raw2inner_id_users, raw2inner_id_items):
        self._ur = ur
        self._ir = ir
        self.n_users = n_users
        self.n_items = n_items
        self.n_ratings = n_ratings
        self.rating_scale = rating_scale
        self.offset = offset
        self._raw2inner_id_users = raw2inner_id_users
        self._raw2inner_id_items = raw2inner_id_items
        self._global_mean = None
        self._inner2raw_id_users = None
        self._inner2raw_id_items = None
        self._csr = None
        self._raw_pos = None  # position of each CSR entry in the raw (insertion) order
        self._dict_built = ur is not None and ir is not None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_csr(cls, row_ptr, items, ratings, n_items, rating_scale=(1, 5), offset=0,
                 raw2inner_id_users=None, raw2inner_id_items=None, raw_pos=None):
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        n_users = len(row_ptr) - 1
        ts = cls(None, None, n_users, int(n_items), int(row_ptr[-1]), rating_scale, offset,
                 raw2inner_id_users if raw2inner_id_users is not None else _IdentityIds(n_users),
                 raw2inner_id_items if raw2inner_id_items is not None else _IdentityIds(n_items))
        ts._csr = (row_ptr, np.ascontiguousarray(items, dtype=np.int32),
                   np.ascontiguousarray(ratings, dtype=np.float64))
        ts._raw_pos = raw_pos
        return ts

    @classmethod
    def from_inner_arrays(cls, uid, iid, ratings, n_users=None, n_items=None, rating_scale=(1, 5),
                          offset=0, raw2inner_id_users=None, raw2inner_id_items=None):
        """Inner ids in insertion order -> CSR in all_ratings() order (stable by user)."""
        uid = np.asarray(uid)
        iid = np.asarray(iid)
        n_users = int(uid.max()) + 1 if n_users is None and len(uid) else (n_users or 0)
        n_items = int(iid.max()) + 1 if n_items is None and len(iid) else (n_items or 0)
        order = np.argsort(uid, kind="stable")
        counts = np.bincount(uid, minlength=n_users)
        row_ptr = np.zeros(n_users + 1, np.int64)
        np.cumsum(counts, out=row_ptr[1:])
        return cls.from_csr(row_ptr, iid[order], np.asarray(ratings, np.float64)[order], n_items,
                            rating_scale, offset, raw2inner_id_users, raw2inner_id_items,
                            raw_pos=order)

    # ------------------------------------------------------------------ array view
    def csr(self):
        """(row_ptr int64[n_users+1], items int32[nnz], ratings float64[nnz]) in all_ratings() order.

        For a dict-built trainset, rows follow user inner ids and each row keeps
        ur[u]'s list order; ``sched_order()`` gives ur's key order."""
        if self._csr is None:
            ur = self._ur
            counts = np.zeros(self.n_users, np.int64)
            for u, lst in ur.items():
                counts[u] = len(lst)
            row_ptr = np.zeros(self.n_users + 1, np.int64)
            np.cumsum(counts, out=row_ptr[1:])
            items = np.empty(row_ptr[-1], np.int32)
            ratings = np.empty(row_ptr[-1], np.float64)
            for u, lst in ur.items():
                if lst:
                    a = np.asarray(lst, dtype=np.float64)
                    items[row_ptr[u]:row_ptr[u + 1]] = a[:, 0].astype(np.int32)
                    ratings[row_ptr[u]:row_ptr[u + 1]] = a[:, 1]
            self._csr = (row_ptr, items, ratings)
        return self._csr

    def sched_order(self):
        """Users in all_ratings() order (= iteration order of ur)."""
        if self._ur is not None:
            return np.fromiter(self._ur.keys(), dtype=np.int32, count=len(self._ur))
        return np.arange(self.n_users, dtype=np.int32)

    # ------------------------------------------------------------------ reference API
    @property
    def ur(self):
        if self._ur is None:
            row_ptr, items, ratings = self._csr
            ur = defaultdict(list)
            il, rl = items.tolist(), ratings.tolist()
            for u in range(self.n_users):
                s, e = int(row_ptr[u]), int(row_ptr[u + 1])
                ur[u] = list(zip(il[s:e], rl[s:e]))
            self._ur = ur
        return self._ur

    @property
    def ir(self):
        if self._ir is None:
            row_ptr, items, ratings = self.csr()
            users = np.repeat(np.arange(self.n_users, dtype=np.int64), np.diff(row_ptr))
            pos = self._raw_pos if self._raw_pos is not None else np.arange(len(items))
            order = np.lexsort((pos, items))  # by item, then raw insertion order
            ir = defaultdict(list)
            ul, rl, il = users[order].tolist(), ratings[order].tolist(), items[order].tolist()
            for x in range(len(il)):
                ir[il[x]].append((ul[x], rl[x]))
            self._ir = ir
        return self._ir

    def csc(self):
        """(item_ptr int64[n_items+1], pos int64[nnz]): for every item, the CSR positions of its
        ratings in ``ir[i]``'s list order (raw insertion order, trainset.py:37-54)."""
        row_ptr, items, _ = self.csr()
        if self._dict_built and self._raw_pos is None:
            # dict-built: follow ir's lists, locating each (u, i) in the CSR
            users = np.repeat(np.arange(self.n_users, dtype=np.int64), np.diff(row_ptr))
            key = users * self.n_items + np.asarray(items, np.int64)
            srt = np.argsort(key, kind="stable")
            pos, ptr = [], [0]
            for i in range(self.n_items):
                for u, _ in self._ir.get(i, []):
                    pos.append(srt[np.searchsorted(key[srt], u * self.n_items + i)])
                ptr.append(len(pos))
            return np.asarray(ptr, np.int64), np.asarray(pos, np.int64)
        pos = self._raw_pos if self._raw_pos is not None else np.arange(len(items))
        order = np.lexsort((pos, items))  # by item, then raw insertion order
        ptr = np.zeros(self.n_items + 1, np.int64)
        np.cumsum(np.bincount(items, minlength=self.n_items), out=ptr[1:])
        return ptr, order.astype(np.int64)

    def knows_user(self, uid):
        """trainset.py:62-74: ``uid in ur``."""
        if self._ur is not None:
            return uid in self._ur
        return isinstance(uid, (int, np.integer)) and 0 <= int(uid) < self.n_users and \
            self._csr[0][int(uid) + 1] > self._csr[0][int(uid)]

    def knows_item(self, iid):
        """trainset.py:76-88: ``iid in ir``."""
        if self._ir is not None:
            return iid in self._ir
        return isinstance(iid, (int, np.integer)) and 0 <= int(iid) < self.n_items

    def to_inner_uid(self, ruid):
        try:
            return self._raw2inner_id_users[ruid]
        except KeyError:
            raise ValueError("User " + str(ruid) + " is not part of the trainset.")

    def to_raw_uid(self, iuid):
        if self._inner2raw_id_users is None:
            self._inner2raw_id_users = {inner: raw for (raw, inner) in
                                        self._raw2inner_id_users.items()}
        try:
            return self._inner2raw_id_users[iuid]
        except KeyError:
            raise ValueError(str(iuid) + " is not a valid inner id.")

    def to_inner_iid(self, riid):
        try:
            return self._raw2inner_id_items[riid]
        except KeyError:
            raise ValueError("Item " + str(riid) + " is not part of the trainset.")

    def to_raw_iid(self, iiid):
        if self._inner2raw_id_items is None:
            self._inner2raw_id_items = {inner: raw for (raw, inner) in
                                        self._raw2inner_id_items.items()}
        try:
            return self._inner2raw_id_items[iiid]
        except KeyError:
            raise ValueError(str(iiid) + " is not a valid inner id.")

    def all_ratings(self):
        """Yield (u, i, r) in the reference order (trainset.py:180-190)."""
        if self._ur is not None:
            for u, u_ratings in self._ur.items():
                for i, r in u_ratings:
                    yield u, i, r
            return
        row_ptr, items, ratings = self._csr
        for u in range(self.n_users):
            for k in range(int(row_ptr[u]), int(row_ptr[u + 1])):
                yield u, int(items[k]), float(ratings[k])

    def build_testset(self):
        return [(self.to_raw_uid(u), self.to_raw_iid(i), r) for (u, i, r) in self.all_ratings()]

    def build_anti_testset(self, fill=None):
        fill = self.global_mean if fill is None else float(fill)
        anti_testset = []
        for u in self.all_users():
            user_items = set([j for (j, _) in self.ur[u]])
            anti_testset += [(self.to_raw_uid(u), self.to_raw_iid(i), fill)
                             for i in self.all_items() if i not in user_items]
        return anti_testset

    def all_users(self):
        return range(self.n_users)

    def all_items(self):
        return range(self.n_items)

    @property
    def global_mean(self):
        """np.mean of all ratings in all_ratings() order (trainset.py:252-261)."""
        if self._global_mean is None:
            if self._ur is not None and self._csr is None:
                self._global_mean = np.mean([r for (_, _, r) in self.all_ratings()])
            else:
                self._global_mean = np.mean(self.csr()[2])
        return self._global_mean
