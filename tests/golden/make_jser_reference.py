"""Collect the JDK-written Java serialization streams the reference's own test resources
hold, as a committed fixture (run from the repo root, in the build container only:
`python tests/golden/make_jser_reference.py`).  Test infrastructure only.

Why these pin the Serializable record length: a Serializable
determinant is `[03]` + the bytes of one `ObjectOutputStream.writeObject` stream with no
length field (SimpleDeterminantEncoder.java:316-341), so its record length is exactly the
length of one stream.  Flink's serializer snapshots write the same kind of stream behind a
big-endian i32 length (TypeSerializerSerializationUtil.java:265-268, the length of the
`ObjectOutputStream` bytes that follow).  Each such prefix is an *independent* statement
of where one JDK-written stream ends: we keep a stream only if the prefix matches the
length the independent Python restatement (oracle/pyref.py jser_len) measures, and the
GPU walker, the C++ oracle and pyref are then pinned to those JDK-written lengths.

Output: tests/golden/jser_reference.json -- a list of {"src": path under the reference,
"off": byte offset of the stream magic in that file, "len": prefix length, "hex": stream}.
Distinct streams only (by content).  The files are data (serializer snapshots, savepoint
metadata) the reference holds; no reference source travels.
"""
from __future__ import annotations

import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyref  # noqa: E402

REF = "/root/reference"
MAGIC = b"\xac\xed\x00\x05"
MAX_FILE = 64 << 20


def scan():
    seen, out = set(), []
    for dirpath, dirnames, files in os.walk(REF):
        dirnames.sort()
        if "/src/test/resources" not in dirpath + "/" and not dirpath.endswith("/src/test/resources"):
            continue
        for fn in sorted(files):
            p = os.path.join(dirpath, fn)
            try:
                if os.path.getsize(p) > MAX_FILE:
                    continue
                data = open(p, "rb").read()
            except OSError:
                continue
            i = data.find(MAGIC)
            while i >= 0:
                if i >= 4:
                    n = struct.unpack(">i", data[i - 4:i])[0]
                    if 5 <= n <= len(data) - i:
                        s = data[i:i + n]
                        if pyref.jser_len(s) == n and s not in seen:
                            seen.add(s)
                            out.append({"src": os.path.relpath(p, REF), "off": i, "len": n, "hex": s.hex()})
                i = data.find(MAGIC, i + 1)
    return out


def main():
    out = scan()
    assert out, "no streams found (is /root/reference present?)"
    path = os.path.join(HERE, "jser_reference.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
        f.write("\n")
    print(f"{len(out)} streams, {sum(x['len'] for x in out)} bytes, max {max(x['len'] for x in out)} -> {path}")


if __name__ == "__main__":
    main()
