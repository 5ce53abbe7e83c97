"""Extract the field constants of every gnark-generated `zp` package in the reference
into tests/golden/fields.json.

Run in the build container only (reads /root/reference as text; nothing is imported or
executed from it).  The output is DATA: modulus q, Limbs, Bits, qInvNeg and rSquare as the
generated code states them, e.g. jindo/internal/zp/element.go:37-72 (q0..q3, qInvNeg) and
:781-789 (rSquare).  The oracle and the HIP library derive these constants themselves; the
tests check the derivations against these values (this pins the Montgomery convention
R = 2^(64*Limbs) and the -q^-1 mod 2^64 constant to the reference's own generated code).

Also records the config-#2 single-word prime p = 47104^4 + 1, which the
reference's jindo-modulus rule would select for `-n 63` (jindo-modulus/main.go:31-71); it has
no generated package in the reference, so its constants are derived (marked derived=True).
"""
import json
import os
import re
import sys

REF = "/root/reference"
PKGS = {
    "jindo_zp": "jindo/internal/zp",
    "zp110": "buckler/internal/zp110",
    "zp220": "buckler/internal/zp220",
    "zp440": "buckler/internal/zp440",
    "zp880": "buckler/internal/zp880",
    "mult_zp": "examples/mult/zp",
    "bfv_zp": "examples/bfv/zp",
}


def parse(path):
    src = open(path).read()
    limbs = int(re.search(r"Limbs\s*=\s*(\d+)", src).group(1))
    bits = int(re.search(r"Bits\s*=\s*(\d+)", src).group(1))
    qhex = re.search(r"q\[base16\]\s*=\s*0x([0-9a-f]+)", src).group(1)
    qinv = int(re.search(r"const qInvNeg\s*=\s*(\d+)", src).group(1))
    m = re.search(r"var rSquare = Uint\{([^}]*)\}", src, re.S)
    r2 = [int(x) for x in re.findall(r"\d+", m.group(1))]
    qlimbs = []
    for i in range(limbs):
        qlimbs.append(int(re.search(r"\bq%d\s*=\s*(\d+)" % i, src).group(1)))
    q = int(qhex, 16)
    assert sum(l << (64 * i) for i, l in enumerate(qlimbs)) == q
    return {"limbs": limbs, "bits": bits, "q_hex": hex(q), "q_le": [str(x) for x in qlimbs],
            "qInvNeg": str(qinv), "rSquare_le": [str(x) for x in r2], "derived": False,
            "source": os.path.relpath(path, REF)}


def main(out):
    fields = {}
    for name, d in PKGS.items():
        fields[name] = parse(os.path.join(REF, d, "element.go"))
    p = 47104 ** 4 + 1
    R = 1 << 64
    fields["p63"] = {"limbs": 1, "bits": p.bit_length(), "q_hex": hex(p), "q_le": [str(p)],
                     "qInvNeg": str((-pow(p, -1, R)) % R), "rSquare_le": [str(R * R % p)],
                     "derived": True, "source": "SURVEY.md 8(d): 47104^4+1 (jindo-modulus rule)"}
    with open(out, "w") as f:
        json.dump(fields, f, indent=1, sort_keys=True)
    print("wrote", out, sorted(fields))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "fields.json"))
