"""Minimal OLE2 + BIFF8 cell reader (test tooling; runs only in the build container).

Purpose: recover the gene-ID order that ``gym_PBN/envs/bittner/utils.py:42-51``
(``pad_ids``) uses to order the nodes of the shipped predictor-set pickles. The
reference reads it with ``pandas.read_excel`` (``bittner/utils.py:35-37``),
which needs ``xlrd`` -- absent from this image. This reader parses the compound
file and the BIFF8 record stream directly; it interprets cell values only
(NUMBER, RK, MULRK, LABELSST, FORMULA numeric results, SST strings) and never
evaluates anything. Its output is pinned by the reference's own expectation in
``tests/test_bittner.py:27`` (the first 70 padded IDs) and ``:18`` (276 weight
IDs); see ``oracle/tools/export_networks.py``.
"""

from __future__ import annotations

import struct

_SIG = bytes.fromhex("D0CF11E0A1B11AE1")
_ENDOFCHAIN = 0xFFFFFFFE
_FREESECT = 0xFFFFFFFF


class _Ole:
    def __init__(self, data: bytes):
        if data[:8] != _SIG:
            raise ValueError("not an OLE2 compound file")
        self.data = data
        self.ssz = 1 << struct.unpack_from("<H", data, 0x1E)[0]
        self.mssz = 1 << struct.unpack_from("<H", data, 0x20)[0]
        n_fat = struct.unpack_from("<I", data, 0x2C)[0]
        dir_start = struct.unpack_from("<I", data, 0x30)[0]
        self.cutoff = struct.unpack_from("<I", data, 0x38)[0]
        minifat_start = struct.unpack_from("<I", data, 0x3C)[0]
        difat_start = struct.unpack_from("<I", data, 0x44)[0]
        difat = list(struct.unpack_from("<109I", data, 0x4C))
        sec = difat_start
        while sec not in (_ENDOFCHAIN, _FREESECT):
            blk = self._sector(sec)
            vals = struct.unpack("<%dI" % (self.ssz // 4), blk)
            difat.extend(vals[:-1])
            sec = vals[-1]
        fat_secs = [s for s in difat if s not in (_ENDOFCHAIN, _FREESECT)][:n_fat]
        fat = []
        for s in fat_secs:
            fat.extend(struct.unpack("<%dI" % (self.ssz // 4), self._sector(s)))
        self.fat = fat
        dir_bytes = self._chain(dir_start)
        self.entries = []
        for off in range(0, len(dir_bytes), 128):
            e = dir_bytes[off:off + 128]
            nlen = struct.unpack_from("<H", e, 0x40)[0]
            name = e[:max(nlen - 2, 0)].decode("utf-16-le", errors="replace")
            etype = e[0x42]
            start = struct.unpack_from("<I", e, 0x74)[0]
            size = struct.unpack_from("<I", e, 0x78)[0]
            self.entries.append((name, etype, start, size))
        root = self.entries[0]
        self.ministream = self._chain(root[2])[: root[3]] if root[2] != _ENDOFCHAIN else b""
        self.minifat = []
        if minifat_start not in (_ENDOFCHAIN, _FREESECT):
            mf = self._chain(minifat_start)
            self.minifat = list(struct.unpack("<%dI" % (len(mf) // 4), mf))

    def _sector(self, s: int) -> bytes:
        off = (s + 1) * self.ssz
        return self.data[off:off + self.ssz]

    def _chain(self, start: int) -> bytes:
        out = []
        s = start
        guard = 0
        while s not in (_ENDOFCHAIN, _FREESECT):
            out.append(self._sector(s))
            s = self.fat[s]
            guard += 1
            if guard > len(self.fat) + 1:
                raise ValueError("FAT cycle")
        return b"".join(out)

    def stream(self, name: str) -> bytes:
        for n, t, start, size in self.entries:
            if n == name and t == 2:
                if size < self.cutoff:
                    out = []
                    s = start
                    while s not in (_ENDOFCHAIN, _FREESECT):
                        off = s * self.mssz
                        out.append(self.ministream[off:off + self.mssz])
                        s = self.minifat[s]
                    return b"".join(out)[:size]
                return self._chain(start)[:size]
        raise KeyError(name)


def _records(wb: bytes, pos: int = 0):
    n = len(wb)
    while pos + 4 <= n:
        rtype, rlen = struct.unpack_from("<HH", wb, pos)
        yield pos, rtype, wb[pos + 4:pos + 4 + rlen]
        pos += 4 + rlen


def _rk(v: int) -> float:
    if v & 2:
        x = float(v >> 2 if not (v & 0x80000000) else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack("<d", struct.pack("<Q", (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


def _parse_sst(chunks):
    """chunks: [SST body, CONTINUE bodies...] -> list[str]."""
    strings = []
    ci, buf = 0, chunks[0]
    pos = 8
    total = struct.unpack_from("<I", buf, 4)[0]

    def need(k):
        nonlocal ci, buf, pos
        if pos + k <= len(buf):
            return
        if pos == len(buf) and ci + 1 < len(chunks):
            ci += 1
            buf, pos = chunks[ci], 0
            return
        raise ValueError("SST field split across CONTINUE")

    while len(strings) < total:
        need(3)
        cch = struct.unpack_from("<H", buf, pos)[0]
        flags = buf[pos + 2]
        pos += 3
        rich = ext = 0
        if flags & 0x08:
            need(2)
            rich = struct.unpack_from("<H", buf, pos)[0]
            pos += 2
        if flags & 0x04:
            need(4)
            ext = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        wide = flags & 1
        chars = []
        left = cch
        while left > 0:
            if pos >= len(buf):
                ci += 1
                buf = chunks[ci]
                wide = buf[0] & 1
                pos = 1
            width = 2 if wide else 1
            take = min(left, (len(buf) - pos) // width)
            seg = buf[pos:pos + take * width]
            chars.append(seg.decode("utf-16-le" if wide else "latin-1"))
            pos += take * width
            left -= take
        strings.append("".join(chars))
        skip = 4 * rich + ext
        while skip > 0:
            if pos >= len(buf):
                ci += 1
                buf, pos = chunks[ci], 0
            t = min(skip, len(buf) - pos)
            pos += t
            skip -= t
    return strings


def read_sheets(path: str) -> dict:
    """Return {sheet_name: {(row, col): value}} for every worksheet."""
    ole = _Ole(open(path, "rb").read())
    try:
        wb = ole.stream("Workbook")
    except KeyError:
        wb = ole.stream("Book")
    sheets = []
    sst_chunks = None
    collecting = False
    for pos, rtype, body in _records(wb):
        if rtype == 0x0085:  # BOUNDSHEET
            off = struct.unpack_from("<I", body, 0)[0]
            cch, flags = body[6], body[7]
            name = body[8:8 + cch * (2 if flags & 1 else 1)].decode("utf-16-le" if flags & 1 else "latin-1")
            sheets.append((name, off))
        elif rtype == 0x00FC:
            sst_chunks = [body]
            collecting = True
        elif rtype == 0x003C and collecting:
            sst_chunks.append(body)
        else:
            collecting = False
        if rtype == 0x000A:  # EOF of workbook globals
            break
    sst = _parse_sst(sst_chunks) if sst_chunks else []
    out = {}
    for name, off in sheets:
        cells = {}
        for pos, rtype, body in _records(wb, off):
            if rtype == 0x000A:
                break
            if rtype == 0x0203:
                r, c = struct.unpack_from("<HH", body, 0)
                cells[(r, c)] = struct.unpack_from("<d", body, 6)[0]
            elif rtype == 0x027E:
                r, c = struct.unpack_from("<HH", body, 0)
                cells[(r, c)] = _rk(struct.unpack_from("<I", body, 6)[0])
            elif rtype == 0x00BD:
                r, c0 = struct.unpack_from("<HH", body, 0)
                n = (len(body) - 6) // 6
                for k in range(n):
                    cells[(r, c0 + k)] = _rk(struct.unpack_from("<I", body, 4 + 6 * k + 2)[0])
            elif rtype == 0x00FD:
                r, c = struct.unpack_from("<HH", body, 0)
                cells[(r, c)] = sst[struct.unpack_from("<I", body, 6)[0]]
            elif rtype == 0x0006:
                r, c = struct.unpack_from("<HH", body, 0)
                res = body[6:14]
                if res[6:8] != b"\xff\xff":
                    cells[(r, c)] = struct.unpack("<d", res)[0]
        out[name] = cells
    return out


def column(cells: dict, col: int, first_row: int):
    rows = sorted(r for (r, c) in cells if c == col and r >= first_row)
    return [cells[(r, col)] for r in rows]


def find_header(cells: dict, text: str, max_row: int = 4):
    for (r, c), v in sorted(cells.items()):
        if r <= max_row and isinstance(v, str) and v.strip() == text:
            return r, c
    raise KeyError(text)
