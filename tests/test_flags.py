import pytest

from distributed_resnet_tensorflow_amd import flags


def _fv(**d):
    fv = flags.FlagValues()
    flags.define_reference_flags(fv, **d)
    return fv


def test_reference_bool_syntaxes():
    fv = _fv()
    fv(["prog", "--sync_replicas=True", "--eval_once", "--nouse_horovod", "--hip_graph=false"])
    assert fv.sync_replicas is True and fv.eval_once is True and fv.use_horovod is False and fv.hip_graph is False
    fv = _fv()
    fv(["prog", "--sync_replicas", "False"])
    assert fv.sync_replicas is False


def test_values_and_defaults():
    fv = _fv(batch_size=128, dataset="imagenet")
    rest = fv(["prog", "--train_steps", "80000", "--log_root=/tmp/x", "--task_index=3", "pos"])
    assert fv.batch_size == 128 and fv.dataset == "imagenet" and fv.train_steps == 80000
    assert fv.log_root == "/tmp/x" and fv.task_index == 3 and rest == ["prog", "pos"]
    assert fv.job_name is None and fv.data_format == "channels_first"


def test_union_flags_present_everywhere():
    # flags that only existed in some reference scripts must parse in every entry point
    fv = _fv()
    fv(["p", "--data_format=channels_last", "--num_epochs=3", "--hidden_units=7", "--replicas_to_aggregate=4",
        "--existing_servers=True", "--ps_hosts=a:1", "--worker_hosts=b:2,c:3", "--job_name=worker"])
    assert fv.hidden_units == 7 and fv.worker_hosts == "b:2,c:3"


def test_unknown_flag_errors():
    with pytest.raises(flags.FlagsError):
        _fv()(["p", "--definitely_not_a_flag=1"])


def test_precision_flag_validation():
    import pytest as _pt
    from distributed_resnet_tensorflow_amd.train.session import make_backend
    assert make_backend("cpu", "fp32").name == "ref"
    assert make_backend("cpu", "bf16").name == "ref"      # CPU: always the fp32 reference backend
    with _pt.raises(ValueError):
        make_backend("cpu", "fp16")


def test_imagenet_entry_defaults_build_resnet50_v2():
    """resnet_imagenet_main.py / resnet_imagenet_eval.py with default flags build the reference's
    ResNet-v2-50 (resnet_model.py:74): --width_multiplier only applies to --model=wide_resnet."""
    from distributed_resnet_tensorflow_amd.cli import entry_flags
    from distributed_resnet_tensorflow_amd.train.trainer import model_spec_from_flags
    for entry in ("imagenet_main", "imagenet_eval_main"):
        spec = model_spec_from_flags(entry_flags(entry, []))
        assert spec.num_params() == 25_551_401, (entry, spec.name)
    F = entry_flags("imagenet_main", ["--model=wide_resnet"])
    assert model_spec_from_flags(F).num_params() == 68_877_609
