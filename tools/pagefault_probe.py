import numpy as np, time
for mb in (67, 537):
    n = mb * 1024 * 1024 // 4
    t0 = time.perf_counter(); a = np.empty(n, np.float32); a[:] = 1.0; t1 = time.perf_counter()
    b = np.empty(n, np.float32); t2 = time.perf_counter(); b[:] = a; t3 = time.perf_counter(); b[:] = a; t4 = time.perf_counter()
    print(f"{mb} MB: first-touch fill {1e3*(t1-t0):.1f} ms, copy into fresh {1e3*(t3-t2):.1f} ms, copy into touched {1e3*(t4-t3):.1f} ms", flush=True)
