"""Flat parameter layouts of the BASELINE models (the SMA path's data format).

Crossbow packs every model variable into one flat fp32 buffer in registration
order (clib-multigpu/model.c:127-157); the SMA step only sees that buffer and
its element count.  These tables give the variable shapes of the two models
BASELINE.json names, so the bench and tests register realistic layouts through
``setModelVariable`` exactly as Model.GPURegister does (Model.java:338-371):

* LeNet (src/test/java/.../LeNet.java:120-170): conv 5x5x32 and 5x5x64 with
  bias, FC 1024 and FC 10 with bias  ->  n = 1,111,946.
* ResNet-50 v1 bottleneck (ResNetv1.java:49,540,632-636,992): convolutions
  without bias, batch-norm gamma/beta, FC 1000 with bias  ->  n = 25,557,032.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

Shape = Tuple[int, ...]


def lenet_variables() -> List[Shape]:
    return [
        (32, 1, 5, 5), (32,),          # conv1 + bias
        (64, 32, 5, 5), (64,),         # conv2 + bias
        (1024, 1024), (1024,),         # fc1 (4*4*64 inputs) + bias
        (10, 1024), (10,),             # fc2 + bias
    ]


def resnet50_variables() -> List[Shape]:
    v: List[Shape] = [(64, 3, 7, 7), (64,), (64,)]  # conv1, bn1 gamma/beta
    inplanes = 64
    for planes, blocks in ((64, 3), (128, 4), (256, 6), (512, 3)):
        for b in range(blocks):
            v += [(planes, inplanes, 1, 1), (planes,), (planes,)]
            v += [(planes, planes, 3, 3), (planes,), (planes,)]
            v += [(planes * 4, planes, 1, 1), (planes * 4,), (planes * 4,)]
            if b == 0:
                v += [(planes * 4, inplanes, 1, 1), (planes * 4,), (planes * 4,)]  # projection shortcut
            inplanes = planes * 4
    v += [(1000, 2048), (1000,)]
    return v


MODELS = {"lenet": lenet_variables, "resnet50": resnet50_variables}

LENET_ELEMENTS = 1_111_946
RESNET50_ELEMENTS = 25_557_032


def elements(shapes: List[Shape]) -> int:
    return int(sum(int(np.prod(s)) for s in shapes))


def register(gpu, shapes: List[Shape], values: np.ndarray = None) -> int:
    """Model.GPURegister: setModel + one setModelVariable(+Buffer) per variable.

    Each variable is registered as op ``k`` order 1; returns the element count.
    """
    n = elements(shapes)
    gpu.setModel(len(shapes), 4 * n)
    off = 0
    for k, s in enumerate(shapes):
        e = int(np.prod(s))
        gpu.setModelVariable(k, 1, list(s), 4 * e)
        if values is not None:
            gpu.setModelVariableBuffer(k, 1, np.ascontiguousarray(values[off:off + e], dtype=np.float32))
        off += e
    return n
