"""Minimal PBM (P4) / PGM (P5) writers and readers used by tests and fixture generation
(test infrastructure; the product's readers are the C++ pbm/pnm drop-ins)."""
import numpy as np


def plane_to_p4_rows(words, cols):
    """uint64 words [rows, wpr] (MSB-first) -> P4 raster bytes (ceil(cols/8) per row)."""
    words = np.ascontiguousarray(words, np.uint64)
    rows = words.shape[0]
    be = words.astype(">u8").view(np.uint8).reshape(rows, -1)
    nb = (cols + 7) // 8
    out = be[:, :nb].copy()
    if cols % 8:
        out[:, -1] &= np.uint8((0xFF << (8 - cols % 8)) & 0xFF)
    return out


def p4_rows_to_plane(raster, rows, cols, wpr=None):
    wpr = wpr or (cols + 63) // 64
    nb = (cols + 7) // 8
    buf = np.zeros((rows, wpr * 8), np.uint8)
    buf[:, :nb] = np.frombuffer(raster, np.uint8, rows * nb).reshape(rows, nb)
    if cols % 8:
        buf[:, nb - 1] &= np.uint8((0xFF << (8 - cols % 8)) & 0xFF)
    return buf.view(">u8").astype(np.uint64).reshape(rows, wpr)


def write_pbm(path, words, cols):
    rows = words.shape[0]
    with open(path, "wb") as f:
        f.write(f"P4\n{cols} {rows}\n".encode())
        f.write(plane_to_p4_rows(words, cols).tobytes())
    return path


def read_pbm_bytes(data):
    """Parse a P4 image written by write_pbm / the reference's write_pbm (pbm.cpp:54-77)."""
    assert data[:2] == b"P4"
    parts = data[2:].split(maxsplit=2)
    cols, rows = int(parts[0]), int(parts[1])
    # header is "P4\n<cols> <rows>\n": exactly one whitespace byte after rows
    hdr = f"P4\n{cols} {rows}\n".encode()
    assert data.startswith(hdr)
    return rows, cols, p4_rows_to_plane(data[len(hdr):], rows, cols)


def write_pgm(path, gray, maxval, comment=None):
    rows, cols = gray.shape
    with open(path, "wb") as f:
        f.write(b"P5\n")
        if comment:
            f.write(f"# {comment}\n".encode())
        f.write(f"{cols} {rows}\n{maxval}\n".encode())
        if maxval < 256:
            f.write(np.ascontiguousarray(gray, np.uint8).tobytes())
        else:
            f.write(np.ascontiguousarray(gray, ">u2").tobytes())
    return path
