"""Minimal read-only HDF5 walker (superblock v0, v1 object headers, symbol-table
groups, contiguous datasets) - enough for Keras 2 weight files. Executes nothing
from the file: it only reads offsets and raw little-endian arrays."""
import struct
import numpy as np


class H5:
    def __init__(self, path):
        self.d = open(path, "rb").read()
        d = self.d
        assert d[:8] == b"\x89HDF\r\n\x1a\n" and d[8] == 0, "superblock v0 only"
        assert d[13] == 8 and d[14] == 8
        # root symbol table entry at 24 + 4*8 = 56
        self.root = self.entry(56)

    def u(self, fmt, off):
        return struct.unpack_from("<" + fmt, self.d, off)

    def entry(self, off):
        name_off, hdr, cache = self.u("QQI", off)
        scratch = self.d[off + 24:off + 40]
        return dict(name_off=name_off, hdr=hdr, cache=cache, scratch=scratch)

    def messages(self, addr):
        d = self.d
        ver, _, nmsg, _, hsize = self.u("BBHII", addr)
        assert ver == 1, ver
        blocks = [(addr + 16, hsize)]
        out = []
        while blocks:
            start, size = blocks.pop(0)
            p = start
            while p + 8 <= start + size and len(out) < nmsg:
                mtype, msize, flags = self.u("HHB", p)
                body = p + 8
                if mtype == 0x10:   # continuation
                    caddr, clen = self.u("QQ", body)
                    blocks.append((caddr, clen))
                out.append((mtype, body, msize))
                p = body + msize
        return out

    def heap_name(self, heap, off):
        assert self.d[heap:heap + 4] == b"HEAP"
        data = self.u("Q", heap + 24)[0]
        s = data + off
        e = self.d.index(b"\0", s)
        return self.d[s:e].decode()

    def group_entries(self, btree, heap):
        d = self.d
        res = []
        def walk(node):
            assert d[node:node + 4] == b"TREE", d[node:node + 4]
            ntype, level, used = self.u("BBH", node + 4)
            p = node + 8 + 16
            kids = []
            for i in range(used):
                p += 8   # key
                kids.append(self.u("Q", p)[0]); p += 8
            for k in kids:
                if level > 0:
                    walk(k)
                else:
                    assert d[k:k + 4] == b"SNOD"
                    n = self.u("H", k + 6)[0]
                    for i in range(n):
                        e = self.entry(k + 8 + 40 * i)
                        res.append((self.heap_name(heap, e["name_off"]), e))
        walk(btree)
        return res

    def children(self, hdr_addr):
        for mtype, body, size in self.messages(hdr_addr):
            if mtype == 0x11:
                bt, hp = self.u("QQ", body)
                return self.group_entries(bt, hp)
        return None

    def dataset(self, hdr_addr):
        shape = dtype = None
        addr = size = None
        for mtype, body, msize in self.messages(hdr_addr):
            if mtype == 0x01:
                ver, rank = self.d[body], self.d[body + 1]
                off = body + (8 if ver == 1 else 4)
                shape = [self.u("Q", off + 8 * i)[0] for i in range(rank)]
            elif mtype == 0x03:
                cls = self.d[body] & 0x0F
                sz = self.u("I", body + 4)[0]
                assert cls == 1, "float datasets only"
                dtype = {4: "<f4", 8: "<f8"}[sz]
            elif mtype == 0x08:
                ver = self.d[body]
                assert ver == 3 and self.d[body + 1] == 1, "contiguous layout v3 only"
                addr, size = self.u("QQ", body + 2)
        a = np.frombuffer(self.d, dtype=dtype, count=int(np.prod(shape)) if shape else 1, offset=addr)
        return a.reshape(shape).copy()

    def walk(self, hdr=None, prefix=""):
        hdr = self.root["hdr"] if hdr is None else hdr
        kids = self.children(hdr)
        if kids is None:
            yield prefix, self.dataset(hdr)
            return
        for name, e in kids:
            yield from self.walk(e["hdr"], prefix + "/" + name)
