"""drn: MI355X-native distributed ResNet training (see README.md)."""
import os as _os

# One hardware queue per HIP stream. HIP's default (GPU_MAX_HW_QUEUES=4) maps the fourth
# normal-priority stream of a process onto a queue another stream already uses, and the two are
# then serialised behind each other's cross-stream waits. The data-parallel step with the ImageNet
# feeder has four (weight-gradient side stream, RCCL's stream, the bucket-report stream, the H2D
# copy stream): its native plan ran 15.0-15.2 ms per step with 4 queues and 10.0 ms with 8, the
# same step without the feeder 9.9-10.0 ms (scripts/imagenet_copy_stream_probe.py,
# profiles/r6_imagenet_copy_stream.jsonl). Read when HIP initialises, so this must precede the
# first GPU call; an explicit setting wins.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
