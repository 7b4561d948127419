import torch, time
from distributed_resnet_tensorflow_amd.models.spec import cifar_resnet_v2, imagenet_resnet_v2
from distributed_resnet_tensorflow_amd.models import oracle
from distributed_resnet_tensorflow_amd.ops.backend import RefBackend
from distributed_resnet_tensorflow_amd.runtime.executor import Executor
torch.manual_seed(0)
for spec, N in [(cifar_resnet_v2(8), 4), (imagenet_resnet_v2(18, num_classes=10, image_size=64), 2), (imagenet_resnet_v2(50, num_classes=10, image_size=64), 2)]:
    ex = Executor(spec, N, RefBackend(), 'cpu', seed=1)
    imgs = torch.randn(N, spec.image_size, spec.image_size, 3)
    ex.images.zero_(); ex.images[..., :3] = imgs
    labels = torch.randint(0, spec.num_classes, (N,))
    ex.labels.copy_(labels.int())
    p = oracle.params_from_store(ex.P)
    st = oracle.state_from_store(ex.P)
    t=time.time()
    ex.forward(train=True); ex.backward()
    t1=time.time()-t
    logits, xent, cost = oracle.loss_fn(spec, p, st, ex.images, labels)
    xent.backward()
    print(spec.name, 'logits err', (logits-ex.logits).abs().max().item(), 'xent', xent.item(), ex.loss_vec.mean().item(), 't', round(t1,2))
    worst = 0
    for s in ex.P.slots:
        g_ex = ex.P.to_tf(s.name, buf=ex.P.grad)
        g_or = p[s.name].grad
        e = ((g_ex-g_or).norm()/(g_or.norm()+1e-12)).item()
        worst=max(worst,e)
        if e > 1e-3: print('  grad mismatch', s.name, e)
    rm_err = max((ex.P.moving(k)[0]-st[k][0]).abs().max().item() for k in st)
    rv_err = max((ex.P.moving(k)[1]-st[k][1]).abs().max().item() for k in st)
    print('  worst grad rel err', worst, 'moving err', rm_err, rv_err)
