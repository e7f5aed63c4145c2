"""Client-frame builder (RFC 6455 §5.2) shared by the golden generator and tests."""
import struct


def frame(opcode, payload, fin=1, key=0x3D21FA37, rsv=0, masked=True, len_form=None):
    """Client frame bytes. len_form forces the 126 / 127 length encodings."""
    n = len(payload)
    b = bytearray([(fin << 7) | (rsv << 4) | opcode])
    m = 0x80 if masked else 0
    form = len_form if len_form else (n if n < 126 else (126 if n <= 65535 else 127))
    if form == 126:
        b += bytes([m | 126]) + struct.pack(">H", n)
    elif form == 127:
        b += bytes([m | 127]) + struct.pack(">Q", n)
    else:
        b += bytes([m | n])
    if masked:
        kb = struct.pack("<I", key)
        b += kb
        b += bytes(c ^ kb[i & 3] for i, c in enumerate(payload))
    else:
        b += payload
    return bytes(b)
