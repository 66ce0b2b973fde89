"""Copy the JSON bench line of a log into profiles/ (measurement tooling): python tools_gpu/save_line.py LOG OUT.json"""
import json
import sys

line = [ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
json.dump(json.loads(line), open(sys.argv[2], "w"), indent=1)
