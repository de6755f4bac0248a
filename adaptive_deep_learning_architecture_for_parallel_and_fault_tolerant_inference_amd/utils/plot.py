"""`plot_model` analogue: the reference renders every configured slice with
`tf.keras.utils.plot_model(md, f"model_{ip}.png")` (`src/node.py:49`).  We write
the Graphviz DOT source (graph/ir.py `Graph.to_dot`) and, when a `dot` binary is
on PATH, render it to the format the file name asks for (.png / .svg / .pdf)."""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Union


def plot_model(model, to_file: str = "model.png", show_shapes: bool = True) -> str:
    """Write `model` (a Model or a Graph) as DOT next to `to_file` and render it if
    Graphviz is installed.  Returns the path written (the rendering, else the .dot)."""
    g = getattr(model, "graph", model)
    base, ext = os.path.splitext(to_file)
    dot_path = base + ".dot"
    os.makedirs(os.path.dirname(os.path.abspath(dot_path)), exist_ok=True)
    with open(dot_path, "w") as f:
        f.write(g.to_dot(show_shapes=show_shapes))
    exe = shutil.which("dot")
    if ext and ext != ".dot" and exe:
        r = subprocess.run([exe, f"-T{ext[1:]}", dot_path, "-o", to_file], capture_output=True)
        if r.returncode == 0:
            return to_file
    return dot_path


def slice_plot_name(directory: str, node_id: Union[str, int], epoch: int) -> str:
    safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in str(node_id))
    return os.path.join(directory, f"model_{safe}_e{epoch}.png")
