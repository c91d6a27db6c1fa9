"""EpisodeBatch / ReplayBuffer with the reference's layout contract and API
(reference: components/episode_buffer.py:6-277).

Every field is a zero-initialised tensor of shape [batch, max_seq_length, *group, *vshape]
(transition data) or [batch, *group, *vshape] (episode-constant data), plus the reserved
int64 `filled` mask.  `update`, slicing and `ReplayBuffer` behave as in the reference.

MI355X-first addition: `time_major=True` stores each transition field as a contiguous
[max_seq_length, batch, ...] buffer and exposes it through a transposed view, so the
tensor a caller sees still has the reference's [batch, time, ...] shape and indexing,
while one time step of all envs (`batch["obs"][:, t]`) is a single contiguous HBM slab:
the HIP env writes it with full-line stores and the agent network reads it with no
gather/copy (`reshape(bs * n, -1)` stays a view).
"""
from types import SimpleNamespace as SN

import numpy as np
import torch


class EpisodeBatch:
    def __init__(self, scheme, groups, batch_size, max_seq_length, data=None, preprocess=None,
                 device="cpu", time_major=False):
        self.scheme = scheme.copy()
        self.groups = groups
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.preprocess = {} if preprocess is None else preprocess
        self.device = device
        self.time_major = time_major
        if data is not None:
            self.data = data
        else:
            self.data = SN(transition_data={}, episode_data={})
            self._setup_data(self.scheme, self.groups, batch_size, max_seq_length, self.preprocess)

    # ---------------------------------------------------------------- allocation
    def _setup_data(self, scheme, groups, batch_size, max_seq_length, preprocess):
        for k, (new_k, transforms) in (preprocess or {}).items():
            assert k in scheme
            vshape, dtype = self.scheme[k]["vshape"], self.scheme[k]["dtype"]
            for tr in transforms:
                vshape, dtype = tr.infer_output_info(vshape, dtype)
            self.scheme[new_k] = {"vshape": vshape, "dtype": dtype}
            for extra in ("group", "episode_const"):
                if extra in self.scheme[k]:
                    self.scheme[new_k][extra] = self.scheme[k][extra]

        assert "filled" not in scheme, '"filled" is a reserved key for masking.'
        scheme.update({"filled": {"vshape": (1,), "dtype": torch.long}})

        for key, info in scheme.items():
            assert "vshape" in info, "Scheme must define vshape for {}".format(key)
            vshape = info["vshape"]
            vshape = (vshape,) if isinstance(vshape, int) else tuple(vshape)
            group = info.get("group", None)
            dtype = info.get("dtype", torch.float32)
            if group:
                assert group in groups, "Group {} must have its number of members defined in _groups_".format(group)
                shape = (groups[group], *vshape)
            else:
                shape = vshape
            if info.get("episode_const", False):
                self.data.episode_data[key] = torch.zeros((batch_size, *shape), dtype=dtype, device=self.device)
            elif self.time_major:
                buf = torch.zeros((max_seq_length, batch_size, *shape), dtype=dtype, device=self.device)
                self.data.transition_data[key] = buf.transpose(0, 1)
            else:
                self.data.transition_data[key] = torch.zeros((batch_size, max_seq_length, *shape), dtype=dtype,
                                                             device=self.device)

    def extend(self, scheme, groups=None):
        self._setup_data(scheme, self.groups if groups is None else groups, self.batch_size,
                         self.max_seq_length, None)

    def to(self, device):
        for store in (self.data.transition_data, self.data.episode_data):
            for k, v in store.items():
                store[k] = v.to(device)
        self.device = device

    def zero_(self):
        """Reset every field to the freshly-allocated state (reuse instead of realloc)."""
        for store in (self.data.transition_data, self.data.episode_data):
            for v in store.values():
                v.zero_()

    # ---------------------------------------------------------------- writes
    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True, preprocess=True):
        """Write `data` at (bs, ts) with scheme dtypes (reference episode_buffer.py:89-129).
        preprocess=False skips the OneHot transform when a fused kernel already wrote it."""
        slices = self._parse_slices((bs, ts))
        for k, v in data.items():
            if k in self.data.transition_data:
                target = self.data.transition_data
                if mark_filled:
                    target["filled"][tuple(slices)] = 1
                    mark_filled = False
                _slices = tuple(slices)
            elif k in self.data.episode_data:
                target = self.data.episode_data
                _slices = slices[0]
            else:
                raise KeyError("{} not found in transition or episode data".format(k))

            dtype = self.scheme[k].get("dtype", torch.float32)
            if isinstance(v, list):
                v = torch.tensor(np.array(v), dtype=dtype, device=self.device)
            dest = target[k][_slices]
            self._check_safe_view(v, dest)
            if str(v.device) != str(dest.device):
                v = v.detach().to(dest.device)
            if v.dtype != dtype:
                v = v.to(dtype)
            target[k][_slices] = v.view_as(dest)

            if preprocess and k in self.preprocess:
                new_k, transforms = self.preprocess[k]
                v = target[k][_slices]
                for tr in transforms:
                    v = tr.transform(v)
                v = v.to(dtype)
                target[new_k][_slices] = v.view_as(target[new_k][_slices])

    def _check_safe_view(self, v, dest):
        idx = len(v.shape) - 1
        for s in dest.shape[::-1]:
            if v.shape[idx] != s:
                if s != 1:
                    raise ValueError("Unsafe reshape of {} to {}".format(v.shape, dest.shape))
            else:
                idx -= 1

    # ---------------------------------------------------------------- reads
    def __getitem__(self, item):
        if isinstance(item, str):
            if item in self.data.episode_data:
                return self.data.episode_data[item]
            if item in self.data.transition_data:
                return self.data.transition_data[item]
            raise ValueError("key {} not in episode or transition data".format(item))
        if isinstance(item, tuple) and all(isinstance(it, str) for it in item):
            new_data = SN(transition_data={}, episode_data={})
            for key in item:
                if key in self.data.transition_data:
                    new_data.transition_data[key] = self.data.transition_data[key]
                elif key in self.data.episode_data:
                    new_data.episode_data[key] = self.data.episode_data[key]
                else:
                    raise KeyError("Unrecognised key {}".format(key))
            new_scheme = {key: self.scheme[key] for key in item}
            new_groups = {self.scheme[key]["group"]: self.groups[self.scheme[key]["group"]]
                          for key in item if "group" in self.scheme[key]}
            return EpisodeBatch(new_scheme, new_groups, self.batch_size, self.max_seq_length, data=new_data,
                                device=self.device, time_major=self.time_major)
        item = self._parse_slices(item)
        new_data = SN(transition_data={}, episode_data={})
        for k, v in self.data.transition_data.items():
            new_data.transition_data[k] = v[tuple(item)]
        for k, v in self.data.episode_data.items():
            new_data.episode_data[k] = v[item[0]]
        ret_bs = self._get_num_items(item[0], self.batch_size)
        ret_t = self._get_num_items(item[1], self.max_seq_length)
        return EpisodeBatch(self.scheme, self.groups, ret_bs, ret_t, data=new_data, device=self.device,
                            time_major=self.time_major)

    @staticmethod
    def _get_num_items(indexing_item, max_size):
        if isinstance(indexing_item, (list, np.ndarray, torch.Tensor)):
            return len(indexing_item)
        if isinstance(indexing_item, slice):
            rng = indexing_item.indices(max_size)
            return 1 + (rng[1] - rng[0] - 1) // rng[2]
        raise TypeError("unsupported index {!r}".format(indexing_item))

    @staticmethod
    def _parse_slices(items):
        if isinstance(items, (slice, int, list, np.ndarray, torch.Tensor)):
            items = (items, slice(None))
        if isinstance(items[1], list):
            raise IndexError("Indexing across Time must be contiguous")
        parsed = []
        for it in items:
            parsed.append(slice(it, it + 1) if isinstance(it, int) else it)
        return parsed

    def max_t_filled(self):
        return torch.sum(self.data.transition_data["filled"], 1).max(0)[0]

    def __repr__(self):
        return "EpisodeBatch. Batch Size:{} Max_seq_len:{} Keys:{} Groups:{}".format(
            self.batch_size, self.max_seq_length, self.scheme.keys(), self.groups.keys())


class ReplayBuffer(EpisodeBatch):
    """Ring buffer of episodes (reference: components/episode_buffer.py:237-277)."""

    def __init__(self, scheme, groups, buffer_size, max_seq_length, preprocess=None, device="cpu"):
        super().__init__(scheme, groups, buffer_size, max_seq_length, preprocess=preprocess, device=device)
        self.buffer_size = buffer_size
        self.buffer_index = 0
        self.episodes_in_buffer = 0

    def insert_episode_batch(self, ep_batch):
        if self.buffer_index + ep_batch.batch_size <= self.buffer_size:
            self.update(ep_batch.data.transition_data,
                        slice(self.buffer_index, self.buffer_index + ep_batch.batch_size),
                        slice(0, ep_batch.max_seq_length), mark_filled=False, preprocess=False)
            self.update(ep_batch.data.episode_data,
                        slice(self.buffer_index, self.buffer_index + ep_batch.batch_size), preprocess=False)
            self.buffer_index += ep_batch.batch_size
            self.episodes_in_buffer = max(self.episodes_in_buffer, self.buffer_index)
            self.buffer_index = self.buffer_index % self.buffer_size
            assert self.buffer_index < self.buffer_size
        else:
            left = self.buffer_size - self.buffer_index
            self.insert_episode_batch(ep_batch[0:left, :])
            self.insert_episode_batch(ep_batch[left:, :])

    def can_sample(self, batch_size):
        return self.episodes_in_buffer >= batch_size

    def sample(self, batch_size, rng=None):
        assert self.can_sample(batch_size)
        if self.episodes_in_buffer == batch_size:
            return self[:batch_size]
        ep_ids = (rng or np.random).choice(self.episodes_in_buffer, batch_size, replace=False)
        return self[ep_ids]

    def __repr__(self):
        return "ReplayBuffer. {}/{} episodes. Keys:{} Groups:{}".format(
            self.episodes_in_buffer, self.buffer_size, self.scheme.keys(), self.groups.keys())
