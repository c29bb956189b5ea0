"""RSCB batch files and the device batch loader.

The reference's input producer (utils/dataset.py:36-75) ends in
``X[N, 13+26]`` float64 with label-encoded ids packed as floats; the models
cast it to float32, so ids are exact only below 2**24.  ``write_criteo`` keeps
the producer's output in the GPU path's layout instead (include/rs_batchio.h:
dense float32, label codes int32/int64, labels, per-field vocab and one-hot
offsets), written and read by native code (csrc/batchio.cpp: mmap, threaded
slab copies).

``DeviceBatchLoader`` streams a file to HBM in chunks of batches: a host
thread copies chunk c+1 from the page cache into a pinned buffer
(rs_cb_read releases the GIL) while one DMA per chunk moves chunk c on a copy
stream; the consumer's stream waits on an event, so H2D overlaps the
kernels.  Batches are ``(dense, ids, labels)`` device tensors, ready for the
models' ``(dense, ids)`` input form.
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading

import numpy as np
import torch

from . import _lib
from .dataset import criteo_compact, features_dict


def _lib_call(name, *args):
    _lib.check(getattr(_lib.lib(), name)(*args), name)


def write_criteo(path, dense, ids, labels=None, field_vocab=None, field_offsets=None, id_dtype=np.int32):
    """Write rows to an RSCB file.  dense [N, nd] (float32 after the cast the
    Keras model applies), ids [N, F] label codes, labels [N]; field_vocab
    defaults to max(id)+1 per field.  Returns the path."""
    dense = np.ascontiguousarray(np.asarray(dense, np.float32))
    ids = np.ascontiguousarray(np.asarray(ids).astype(id_dtype))
    N = dense.shape[0]
    if ids.shape[0] != N:
        raise ValueError("dense and ids must have the same number of rows")
    if field_vocab is None:
        field_vocab = ids.max(axis=0).astype(np.int64) + 1 if N else np.ones(ids.shape[1], np.int64)
    vocab = np.ascontiguousarray(np.asarray(field_vocab, np.int64))
    offs = None if field_offsets is None else np.ascontiguousarray(np.asarray(field_offsets, np.int64))
    lab = None if labels is None else np.ascontiguousarray(np.asarray(labels, np.float32))
    _lib_call("rs_cb_write", os.fsencode(str(path)), N, dense.shape[1], ids.shape[1], ids.dtype.itemsize,
              dense.ctypes.data, ids.ctypes.data, None if lab is None else lab.ctypes.data, vocab.ctypes.data,
              None if offs is None else offs.ctypes.data)
    return path


def criteo_txt_to_rscb(txt_path, out_path, id_dtype=np.int32):
    """The reference's producer (fillna, MinMaxScaler, LabelEncoder; vocab =
    features_dict's nunique()+1) over a Criteo text file, straight to RSCB —
    no float-packed ids, no one-hot matrix."""
    dense, ids, label, _ = criteo_compact(txt_path)
    vocab = [f["feat_onehot_dim"] for f in features_dict(txt_path)[1]]
    return write_criteo(out_path, dense, ids, label, vocab, id_dtype=id_dtype)


class RSCBFile:
    """An open (mmapped) RSCB file."""

    def __init__(self, path):
        h = _lib.lib().rs_cb_open(os.fsencode(str(path)))
        if not h:
            raise OSError(_lib.lib().rs_last_error_string().decode())
        self._h = h
        n, nd, nf, ib = C.c_int64(), C.c_int(), C.c_int(), C.c_int()
        _lib_call("rs_cb_info", h, C.byref(n), C.byref(nd), C.byref(nf), C.byref(ib), None, None)
        self.n_rows, self.n_dense, self.n_sparse, self.id_bytes = n.value, nd.value, nf.value, ib.value
        self.field_vocab = np.zeros(self.n_sparse, np.int64)
        self.field_offsets = np.zeros(self.n_sparse, np.int64)
        _lib_call("rs_cb_info", h, None, None, None, None, self.field_vocab.ctypes.data,
                  self.field_offsets.ctypes.data)
        self.id_dtype = np.int32 if self.id_bytes == 4 else np.int64

    def read_into(self, row0, count, dense=None, ids=None, labels=None):
        """Copy rows [row0, row0+count) into host buffers (numpy arrays or
        CPU tensors, contiguous; any may be None)."""
        p = lambda a: None if a is None else (a.data_ptr() if torch.is_tensor(a) else a.ctypes.data)
        _lib_call("rs_cb_read", self._h, row0, count, p(dense), p(ids), p(labels))

    def read(self, row0=0, count=None):
        count = self.n_rows - row0 if count is None else count
        dense = np.empty((count, self.n_dense), np.float32)
        ids = np.empty((count, self.n_sparse), self.id_dtype)
        labels = np.empty(count, np.float32)
        self.read_into(row0, count, dense, ids, labels)
        return dense, ids, labels

    def close(self):
        if self._h:
            _lib.lib().rs_cb_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class DeviceBatchLoader:
    """Iterate an RSCB file in batches of ``batch`` rows as device tensors
    (dense f32 [B, nd], ids [B, F] int32/int64, labels f32 [B]); the tail
    batch is smaller.

    Rows move in chunks of ``group`` batches: one persistent host thread
    copies a chunk's three slabs from the page cache into ONE pinned buffer
    (rs_cb_read, threaded, GIL released), one DMA moves the whole buffer to
    HBM on ``copy_stream``, and the consumer's stream waits on its event.
    ``depth`` chunk slots rotate, so reading chunk c+1, copying chunk c and
    the kernels on chunk c-1 overlap.  A yielded batch stays valid until the
    loader has moved ``depth - 1`` chunks further."""

    def __init__(self, file, batch, device=None, depth=3, group=16):
        self.file = file if isinstance(file, RSCBFile) else RSCBFile(file)
        self.batch = int(batch)
        self.group = max(1, int(group))
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.depth = max(2, int(depth))
        f = self.file
        R = self.batch * self.group  # rows per chunk
        self._rows = R
        # byte layout of a chunk buffer: [dense R*nd*4 | ids R*F*ib | labels R*4], 16-B aligned parts
        al = lambda x: (x + 15) // 16 * 16
        self._o_ids = al(R * f.n_dense * 4)
        self._o_lab = al(self._o_ids + R * f.n_sparse * f.id_bytes)
        nbytes = al(self._o_lab + R * 4)
        self._host = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(self.depth)]
        self._dev = [torch.empty(nbytes, dtype=torch.uint8, device=self.device) for _ in range(self.depth)]
        self.copy_stream = torch.cuda.Stream(self.device)
        self._done = [None] * self.depth  # event: the slot's H2D finished (pinned buffer free)
        self._tid = torch.int32 if f.id_bytes == 4 else torch.int64

    def __len__(self):
        return (self.file.n_rows + self.batch - 1) // self.batch

    def _views(self, buf, n):
        f = self.file
        dense = buf[:n * f.n_dense * 4].view(torch.float32).view(n, f.n_dense)
        ids = buf[self._o_ids:self._o_ids + n * f.n_sparse * f.id_bytes].view(self._tid).view(n, f.n_sparse)
        lab = buf[self._o_lab:self._o_lab + n * 4].view(torch.float32)
        return dense, ids, lab

    def _fill(self, c):
        """Chunk c -> its pinned slot; returns its row count."""
        f = self.file
        row0 = c * self._rows
        n = min(self._rows, f.n_rows - row0)
        h = self._host[c % self.depth]
        base = h.data_ptr()
        _lib_call("rs_cb_read", self.file._h, row0, n, base, base + self._o_ids, base + self._o_lab)
        return n

    def __iter__(self):
        f = self.file
        n_chunks = (f.n_rows + self._rows - 1) // self._rows
        if n_chunks == 0:
            return
        consumer = torch.cuda.current_stream(self.device)
        reuse = [None] * self.depth  # event: the consumer is done with the slot's device buffer
        jobs, results = queue.Queue(), queue.Queue()

        def worker():
            while True:
                c = jobs.get()
                if c is None:
                    return
                try:
                    results.put((c, self._fill(c), None))
                except Exception as e:  # noqa: BLE001 - re-raised in the consumer
                    results.put((c, 0, e))

        th = threading.Thread(target=worker, daemon=True)
        th.start()
        try:
            jobs.put(0)
            for c in range(n_chunks):
                slot = c % self.depth
                cc, n, err = results.get()
                if err is not None:
                    raise err
                assert cc == c
                if c + 1 < n_chunks:
                    nxt = (c + 1) % self.depth
                    if self._done[nxt] is not None:
                        self._done[nxt].synchronize()  # the pinned slot's last H2D has finished
                    jobs.put(c + 1)
                with torch.cuda.stream(self.copy_stream):
                    if reuse[slot] is not None:
                        self.copy_stream.wait_event(reuse[slot])
                    nb = self._o_lab + n * 4
                    self._dev[slot][:nb].copy_(self._host[slot][:nb], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                    self._done[slot] = ev
                consumer.wait_event(ev)
                dense, ids, lab = self._views(self._dev[slot], self._rows)
                for r0 in range(0, n, self.batch):
                    r1 = min(n, r0 + self.batch)
                    yield dense[r0:r1], ids[r0:r1], lab[r0:r1]
                r = torch.cuda.Event()
                r.record(consumer)
                reuse[slot] = r
        finally:
            jobs.put(None)
            th.join()
        torch.cuda.current_stream(self.device).synchronize()
