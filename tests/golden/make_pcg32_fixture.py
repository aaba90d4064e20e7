"""Regenerate tests/golden/pcg32_demo.json from the reference's known-answer
output ext/pcg32/pcg32-demo.out (seed 42/54, five rounds).  Run in the build
container (the reference checkout is not present on the GPU box)."""
import json
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/ext/pcg32/pcg32-demo.out"
text = open(src).read()
rounds = []
for block in re.split(r"Round \d+:", text)[1:]:
    u32 = [int(x, 16) for x in re.search(r"32bit:(.*)", block).group(1).split()]
    coins = re.search(r"Coins: (\S+)", block).group(1)
    rolls = [int(x) for x in re.search(r"Rolls:(.*)", block).group(1).split()]
    cards = re.search(r"Cards: (.*?)(?:\n\s*\n|\Z)", block, re.S).group(1).split()
    rounds.append({"u32": u32, "coins": coins, "rolls": rolls, "cards": cards})
json.dump({"seed": [42, 54], "source": "ext/pcg32/pcg32-demo.out", "rounds": rounds},
          open(__file__.replace("make_pcg32_fixture.py", "pcg32_demo.json"), "w"), indent=1)
print(len(rounds), "rounds")
