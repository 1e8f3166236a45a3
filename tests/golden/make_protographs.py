"""Extract the IEEE 802.11n / 802.16 protograph tables into
ldpc_sparc_amd/data/protographs.json (standard data, the tables of
ldpc_jossy/py/ldpc.py:assign_proto :24-272).

Build-container script: reads the reference through ref_harness; the product
only reads the committed JSON.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ref_harness  # noqa: E402

OUT = os.path.join(ref_harness.REPO, "ldpc_sparc_amd", "data", "protographs.json")


def main():
    ldpc = ref_harness.import_reference()[0]
    rates = ["1/2", "2/3", "3/4", "5/6"]
    data = {"802.16": {}, "802.11n": {}}
    for rate in rates:
        for ptype in (["A", "B"] if rate in ("2/3", "3/4") else ["A"]):
            c = ldpc.code("802.16", rate, 27, ptype)
            data["802.16"].setdefault(rate, {})[ptype] = c.proto.tolist()
    for z in (27, 54, 81):
        for rate in rates:
            c = ldpc.code("802.11n", rate, z, "A")
            data["802.11n"].setdefault(str(z), {})[rate] = c.proto.tolist()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        f.write("{\n")
        parts = []
        for std, d in data.items():
            lines = []
            for k1, d1 in d.items():
                inner = []
                for k2, proto in d1.items():
                    rows = ",\n        ".join(json.dumps(r) for r in proto)
                    inner.append(f'      "{k2}": [\n        {rows}]')
                lines.append(f'    "{k1}": {{\n' + ",\n".join(inner) + "}")
            parts.append(f'  "{std}": {{\n' + ",\n".join(lines) + "}")
        f.write(",\n".join(parts) + "\n}\n")
    json.load(open(OUT))  # validate
    print("wrote", OUT)


if __name__ == "__main__":
    main()
