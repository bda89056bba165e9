#!/usr/bin/env python3
"""Write the Ur5Sih observable registration table (data) used by handarm_hip/observables.py.

Reads the reference's ``register_observables`` (tasks/hand_arm/base/ur5sih.py:233-345, then
tasks/hand_arm/env/multi_object.py:121-417, which calls super() first) as text with ``ast`` and records, in
registration order, each observable's name, ``required`` flag and ``requires`` list. That is the input of the
reference's ``ActiveObservables.sort`` (utils/observables.py:219-257), which handarm_hip/observables.py
restates. Build container only (reads /root/reference); the JSON it writes is committed.
"""
import ast
import json
import os

REF = "/root/reference/isaacgymenvs/tasks/hand_arm"
FILES = [os.path.join(REF, "base/ur5sih.py"), os.path.join(REF, "env/multi_object.py")]
OUT = os.path.join(os.path.dirname(__file__), "..", "..", "isaacgym-hand-arm_amd", "handarm_hip", "assets",
                   "ur5sih_observables.json")


def registered_observables():
    out = []
    for fi, path in enumerate(FILES):
        tree = ast.parse(open(path).read())
        for fn in ast.walk(tree):
            if not (isinstance(fn, ast.FunctionDef) and fn.name == "register_observables"):
                continue
            for node in ast.walk(fn):
                if not (isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "register_observable"):
                    continue
                kw = {k.arg: k.value for k in node.args[0].keywords}
                if not isinstance(kw.get("name"), ast.Constant):
                    continue            # camera observables (f-string names): not built here
                required = bool(kw["required"].value) if "required" in kw else False
                requires = [e.value for e in kw["requires"].elts] if "requires" in kw else []
                out.append(((fi, node.lineno), {"name": kw["name"].value, "required": required,
                                                "requires": requires,
                                                "source": f"{os.path.relpath(path, REF)}:{node.lineno}"}))
    return [o[1] for o in sorted(out, key=lambda o: o[0])]


if __name__ == "__main__":
    table = registered_observables()
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_observables_table.py", "observables": table}, f, indent=1)
    print(len(table), "observables ->", OUT)
