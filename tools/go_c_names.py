#!/usr/bin/env python3
"""Inventory of the SWIG names the reference's Go code binds from package `c` -- the server side
(src/server/*.go, src/server_util/*.go) and the client and benchmark that build against the same
package (src/client/*.go, src/benchmark/*.go) -- mapped to the C declarations a drop-in library must
provide (src/c/c.swigcxx:15-24 wraps the headers with SWIG in C++ mode).

SWIG's Go naming: a function f is exported as F (first letter upper-cased); a global variable
G gets the accessors GetG / SetG; a struct type s is the Go type S with NewS / DeleteS.

    python tools/go_c_names.py [/root/reference/src] > tests/golden/go_c_names.json

Needs the reference sources (this container only); the JSON it prints is committed and read by
tests/test_abi.py::test_header_declares_every_go_bound_name.
"""
import json
import os
import re
import sys


def main(argv):
    src = argv[1] if len(argv) > 1 else "/root/reference/src"
    names = {}
    for sub in ("server", "server_util", "client", "benchmark"):
        d = os.path.join(src, sub)
        for f in sorted(os.listdir(d)):
            if not f.endswith(".go"):
                continue
            text = open(os.path.join(d, f)).read()
            for i, line in enumerate(text.splitlines(), 1):
                # names in comments too (e.g. hollanti.go:20 `//q := c.Choose(...)`): declaring
                # them costs nothing and keeps a commented call compilable if restored
                for m in re.finditer(r"\bc\.([A-Z][A-Za-z0-9_]*)", line):
                    names.setdefault(m.group(1), []).append(f"src/{sub}/{f}:{i}")
    out = []
    for go, sites in sorted(names.items()):
        if go.startswith("Get") and go[3:].isupper() or go.startswith("Get") and "_" in go:
            kind, c = "global", go[3:]
        elif go.startswith("New") or go.startswith("Delete"):
            kind, c = "ctor", (go[3:] if go.startswith("New") else go[6:]).lower()
        elif go in ("Server", "Client"):
            kind, c = "type", go.lower()
        else:
            kind, c = "function", go[0].lower() + go[1:]
        out.append({"go": go, "kind": kind, "c": c, "sites": sites[:3]})
    json.dump({"source": "src/{server,server_util,client,benchmark}/*.go", "names": out}, sys.stdout,
              indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv)
