import time, torch, sys
sys.path.insert(0, '.')
from truth_recommendation_gnn_amd import minibatch
dev = torch.device('cuda')
U, P, E, B = 9_000_000, 1_000_000, 20_000_000, 1024
g = torch.Generator(device=dev).manual_seed(0)
ei = torch.stack([torch.randint(0, U, (E,), device=dev, generator=g), torch.randint(0, P, (E,), device=dev, generator=g)])
ll = minibatch.LinkLoss(B, B, 2 * B, dev)
def timeit(fn, n=200):
    for _ in range(10): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    return (t1 - t) / n * 1e6, (t2 - t) / n * 1e6
ids = torch.randint(0, E, (B,), device=dev, generator=g)
lb = minibatch.link_batch(ei, ids, P, generator=g)
print('link_batch host/total us', timeit(lambda: minibatch.link_batch(ei, ids, P, generator=g)))
print('LinkLoss.load host/total us', timeit(lambda: ll.load(lb.pu, lb.pp, lb.pn)))
print('argsort stable host/total us', timeit(lambda: torch.argsort(lb.pu, stable=True)))
print('argsort host/total us', timeit(lambda: torch.argsort(lb.pu)))
print('unique host/total us', timeit(lambda: torch.unique(lb.pos_u)))
print('sort host/total us', timeit(lambda: torch.sort(lb.pu, stable=True)))
