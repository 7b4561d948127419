"""ResNet v2 (pre-activation) topology specs with TensorFlow-1 variable naming.

One declarative description of the network drives the pure-PyTorch oracle
(``models.oracle``), the static-plan executor (``runtime.executor``), the parameter/FLOP
report (``models.analysis``) and the TensorBundle checkpoint layout (``ckpt``).

Reference semantics reproduced here (resnet_model_official.py):
  * CIFAR 6n+2 generator (:217-278): stem conv3x3/1 -> 16; three stages of n building blocks
    with 16/32/64 filters, strides 1/2/2; final BN-ReLU; global average pool; dense.
  * ImageNet generator (:281-366): stem conv7x7/2 -> 64; max-pool 3x3/2 SAME; four stages
    (64/128/256/512 filters, strides 1/2/2/2) of building (18/34) or bottleneck (50..200)
    blocks; final BN-ReLU; global average pool; dense (1001 classes for ImageNet).
  * The FIRST block of every stage has a 1x1 projection shortcut on the BN-ReLU output, even
    when the shape does not change (:202-209); the stride sits on the 3x3 conv (:166-168).
  * Stride>1 convs use fixed padding ((k-1)//2 before, the rest after) + VALID; stride-1 convs
    use SAME (:53-91). No conv bias.
  * tf.layers auto-naming in creation order: conv2d, conv2d_1, ...; batch_normalization,
    batch_normalization_1, ...; dense. Inside a block the creation order is
    BN1 -> (projection conv) -> conv1 -> BN2 -> conv2 [-> BN3 -> conv3] (:113-130, :153-175).

Extension (not in the reference, labelled as such): ``wide_resnet_50_2`` doubles the bottleneck
inner width (Wide ResNet paper cited in reference README.md:110-112).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class Conv:
    name: str           # TF scope, e.g. "conv2d_3" -> variable "conv2d_3/kernel"
    cin: int
    cout: int
    k: int
    stride: int
    cin_store: int = 0  # channels as stored/computed (stem input padded 3 -> 8); 0 = cin

    def __post_init__(self):
        if not self.cin_store:
            self.cin_store = self.cin

    @property
    def pad(self) -> int:
        """Leading pad: SAME for stride 1, fixed_padding (k-1)//2 for stride > 1 (same value for odd k)."""
        return (self.k - 1) // 2

    def out_hw(self, h: int) -> int:
        if self.stride == 1:
            return h
        total = self.k - 1
        return (h + total - self.k) // self.stride + 1

    @property
    def params(self) -> int:
        return self.k * self.k * self.cin * self.cout


@dataclass
class BN:
    name: str  # "batch_normalization_7"
    c: int


@dataclass
class Block:
    kind: str                 # "basic" | "bottleneck"
    stage: int
    index: int
    in_c: int
    out_c: int
    in_hw: int
    out_hw: int
    stride: int
    bn1: BN
    proj: Optional[Conv]
    convs: List[Conv]         # basic: [conv3x3(stride), conv3x3]; bottleneck: [1x1, 3x3(stride), 1x1]
    bns: List[BN]             # BNs preceding convs[1:], i.e. bn2 (and bn3)


@dataclass
class NetSpec:
    name: str
    dataset: str
    num_classes: int
    image_size: int
    in_channels: int          # 3 (stored as 8)
    stem: Conv
    stem_hw: int              # spatial size after the stem conv
    maxpool: bool             # ImageNet 3x3/2 SAME max-pool after the stem
    pool_hw: int              # spatial size entering stage 1
    blocks: List[Block] = field(default_factory=list)
    final_bn: Optional[BN] = None
    final_hw: int = 0
    final_c: int = 0
    dense_name: str = "dense"

    # -- TF variable inventory, creation order ---------------------------------------------------
    def trainable_variables(self):
        """[(tf_name, tf_shape, kind, owner)] in tf.trainable_variables() order."""
        out = []

        def conv(c: Conv):
            out.append((f"{c.name}/kernel", (c.k, c.k, c.cin, c.cout), "conv", c))

        def bn(b: BN):
            out.append((f"{b.name}/gamma", (b.c,), "gamma", b))
            out.append((f"{b.name}/beta", (b.c,), "beta", b))

        conv(self.stem)
        for blk in self.blocks:
            bn(blk.bn1)
            if blk.proj is not None:
                conv(blk.proj)
            conv(blk.convs[0])
            for b, c in zip(blk.bns, blk.convs[1:]):
                bn(b)
                conv(c)
        bn(self.final_bn)
        out.append((f"{self.dense_name}/kernel", (self.final_c, self.num_classes), "dense_w", None))
        out.append((f"{self.dense_name}/bias", (self.num_classes,), "dense_b", None))
        return out

    def batch_norms(self) -> List[BN]:
        bns = []
        for blk in self.blocks:
            bns.append(blk.bn1)
            bns.extend(blk.bns)
        bns.append(self.final_bn)
        return bns

    def convs(self) -> List[Conv]:
        cs = [self.stem]
        for blk in self.blocks:
            if blk.proj is not None:
                cs.append(blk.proj)
            cs.extend(blk.convs)
        return cs

    def num_params(self) -> int:
        n = 0
        for _, shape, _, _ in self.trainable_variables():
            p = 1
            for d in shape:
                p *= d
            n += p
        return n

    def forward_flops(self) -> int:
        """Multiply-add FLOPs (x2) of one image's forward pass: convs + dense."""
        fl = 0
        hw = self.image_size
        fl += 2 * self.stem.params * self.stem_hw * self.stem_hw
        for blk in self.blocks:
            if blk.proj is not None:
                fl += 2 * blk.proj.params * blk.out_hw * blk.out_hw
            h = blk.in_hw
            for c in blk.convs:
                h = c.out_hw(h)
                fl += 2 * c.params * h * h
        fl += 2 * self.final_c * self.num_classes
        del hw
        return fl


class _Namer:
    def __init__(self):
        self.conv = 0
        self.bn = 0

    def next_conv(self) -> str:
        n = "conv2d" if self.conv == 0 else f"conv2d_{self.conv}"
        self.conv += 1
        return n

    def next_bn(self) -> str:
        n = "batch_normalization" if self.bn == 0 else f"batch_normalization_{self.bn}"
        self.bn += 1
        return n


def _stage(spec: NetSpec, nm: _Namer, kind: str, stage: int, filters: int, blocks: int, stride: int,
           in_c: int, hw: int, width: int = 1) -> tuple[int, int]:
    out_c = filters * 4 if kind == "bottleneck" else filters
    for i in range(blocks):
        s = stride if i == 0 else 1
        bn1 = BN(nm.next_bn(), in_c)
        proj = Conv(nm.next_conv(), in_c, out_c, 1, s) if i == 0 else None
        convs, bns = [], []
        if kind == "basic":
            c1 = Conv(nm.next_conv(), in_c, filters, 3, s)
            b2 = BN(nm.next_bn(), filters)
            c2 = Conv(nm.next_conv(), filters, filters, 3, 1)
            convs, bns = [c1, c2], [b2]
        else:
            mid = filters * width
            c1 = Conv(nm.next_conv(), in_c, mid, 1, 1)
            b2 = BN(nm.next_bn(), mid)
            c2 = Conv(nm.next_conv(), mid, mid, 3, s)
            b3 = BN(nm.next_bn(), mid)
            c3 = Conv(nm.next_conv(), mid, out_c, 1, 1)
            convs, bns = [c1, c2, c3], [b2, b3]
        out_hw = convs[0].out_hw(hw) if kind == "basic" else convs[1].out_hw(hw)
        spec.blocks.append(Block(kind, stage, i, in_c, out_c, hw, out_hw, s, bn1, proj, convs, bns))
        in_c, hw = out_c, out_hw
    return in_c, hw


def cifar_resnet_v2(resnet_size: int = 50, num_classes: int = 10) -> NetSpec:
    """cifar10_resnet_v2_generator (reference resnet_model_official.py:217-278)."""
    if resnet_size % 6 != 2:
        raise ValueError(f"resnet_size must be 6n + 2: {resnet_size}")
    n = (resnet_size - 2) // 6
    nm = _Namer()
    stem = Conv(nm.next_conv(), 3, 16, 3, 1, cin_store=8)
    spec = NetSpec(f"cifar_resnet{resnet_size}_v2", "cifar", num_classes, 32, 3, stem, 32, False, 32)
    c, hw = 16, 32
    for stage, (f, s) in enumerate(((16, 1), (32, 2), (64, 2)), start=1):
        c, hw = _stage(spec, nm, "basic", stage, f, n, s, c, hw)
    spec.final_bn = BN(nm.next_bn(), c)
    spec.final_hw, spec.final_c = hw, c
    return spec


IMAGENET_SIZES = {
    18: ("basic", [2, 2, 2, 2]),
    34: ("basic", [3, 4, 6, 3]),
    50: ("bottleneck", [3, 4, 6, 3]),
    101: ("bottleneck", [3, 4, 23, 3]),
    152: ("bottleneck", [3, 8, 36, 3]),
    200: ("bottleneck", [3, 24, 36, 3]),
}


def imagenet_resnet_v2(resnet_size: int = 50, num_classes: int = 1001, width: int = 1,
                       image_size: int = 224) -> NetSpec:
    """imagenet_resnet_v2 (reference resnet_model_official.py:281-366); width=2 -> WRN-50-2 (extension)."""
    if resnet_size not in IMAGENET_SIZES:
        raise ValueError(f"Not a valid resnet_size: {resnet_size}")
    kind, layers = IMAGENET_SIZES[resnet_size]
    nm = _Namer()
    stem = Conv(nm.next_conv(), 3, 64, 7, 2, cin_store=8)
    stem_hw = stem.out_hw(image_size)
    pool_hw = (stem_hw + 1) // 2  # max_pooling2d(3, 2, 'SAME')
    tag = f"wide_resnet{resnet_size}_{width}" if width != 1 else f"imagenet_resnet{resnet_size}_v2"
    spec = NetSpec(tag, "imagenet", num_classes, image_size, 3, stem, stem_hw, True, pool_hw)
    c, hw = 64, pool_hw
    for stage, (f, s) in enumerate(((64, 1), (128, 2), (256, 2), (512, 2)), start=1):
        c, hw = _stage(spec, nm, kind, stage, f, layers[stage - 1], s, c, hw, width=width)
    spec.final_bn = BN(nm.next_bn(), c)
    spec.final_hw, spec.final_c = hw, c
    return spec


def build_spec(dataset: str, resnet_size: int | None = None, model: str = "resnet", width: int = 1,
               num_classes: int | None = None) -> NetSpec:
    """Network selection of the reference ResNet wrapper (resnet_model.py:71-74, size fixed to 50
    there; `--resnet_size` makes it selectable here). cifar100 is supported."""
    if model == "wide_resnet":
        width = max(width, 2)
    if dataset in ("cifar10", "cifar100", "cifar"):
        nc = num_classes or (100 if dataset == "cifar100" else 10)
        return cifar_resnet_v2(resnet_size or 50, nc)
    if dataset == "imagenet":
        return imagenet_resnet_v2(resnet_size or 50, num_classes or 1001, width=width)
    raise ValueError(f"unknown dataset {dataset}")
