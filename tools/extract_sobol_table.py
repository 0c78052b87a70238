"""Extract the Sobol direction-number table (128 uint32) from the reference's HalogenRandom.hlsl:10-46 into
tests/golden/sobol_table.json — a data fixture the oracle's Joe–Kuo-constructed table is checked against.
Runs only in the build container (the reference is not on the GPU box)."""
import json
import re
from pathlib import Path

SRC = Path("/root/reference/Assets/Scripts/Halogen Shaders/HalogenRandom.hlsl")
text = SRC.read_text()
body = text[text.index("sobol_table[128]"):]
body = body[body.index("{") + 1: body.index("};")]
vals = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", body)]
assert len(vals) == 128, len(vals)
out = Path(__file__).resolve().parents[1] / "tests" / "golden" / "sobol_table.json"
out.write_text(json.dumps({"source": "HalogenRandom.hlsl:10-46", "dims": 4, "bits": 32,
                           "table": [vals[d * 32:(d + 1) * 32] for d in range(4)]}, indent=1))
print("wrote", out)
