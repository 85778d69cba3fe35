"""Fixture: real ENet wire datagrams.

Runs oracle/_ref/loopback_ref -- live ENet hosts built from the reference
sources with compress.c and enet_crc32 enabled -- with ENET_LOOPBACK_DUMP, so
its intercept hook records every received datagram as it was on the wire plus
the checksum seed protocol.c uses for it.  Each record keeps the wire bytes,
the seed, and the datagram protocol.c goes on to parse (oracle restatement of
protocol.c:1022-1091 with the reference compress.c and enet_crc32).  The
script checks that every recorded datagram passes the checksum, and that
re-encoding it (protocol.c:1686-1718) gives back the exact wire bytes.

usage: python tests/golden/make_dgram_golden.py   (needs /root/reference at build time)
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def main():
    from oracle.pyoracle import Coder, datagram_decode, datagram_encode
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
    ref = Coder("reference")
    cases = []
    for checksum, port, count in ((1, 47811, 160), (0, 47813, 80)):
        with tempfile.NamedTemporaryFile(suffix=".jsonl", delete=False) as f:
            path = f.name
        env = dict(os.environ, ENET_LOOPBACK_DUMP=path, ENET_LOOPBACK_CHECKSUM=str(checksum))
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "loopback_ref"), "both", str(port), str(count)],
                           env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        for line in open(path):
            rec = json.loads(line)
            wire = bytes.fromhex(rec["wire"])
            dec = datagram_decode(wire, bool(rec["checksum"]), rec["seed"], ref)
            assert dec, "a real datagram failed the restated receive path"
            assert datagram_encode(dec, bool(rec["checksum"]), rec["seed"], ref) == wire
            cases.append({"checksum": rec["checksum"], "seed": rec["seed"], "wire": rec["wire"],
                          "decoded": dec.hex(), "compressed": bool(wire[0] & 0x40)})
        os.unlink(path)
    out = os.path.join(HERE, "dgram_cases.json")
    with open(out, "w") as f:
        json.dump({"source": "oracle/_ref/loopback_ref (reference protocol.c + compress.c + enet_crc32)",
                   "cases": cases}, f)
    print(len(cases), "datagrams,", sum(c["compressed"] for c in cases), "compressed ->", out)


if __name__ == "__main__":
    main()
