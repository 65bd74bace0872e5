import sys, numpy as np
sys.path.insert(0, 'tests')
from _pkg import load_pkg, load_oracle
from _scenes import sequence
from _vocab import vocabulary
pkg = load_pkg()
path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
voc = pkg.ORBVocabulary(path)
cfg, traj, frames = sequence(3, 90)
tr = pkg.Tracker(pkg.OrbParams(1000, 1.2, 8, 20, 7), pkg.make_camera(cfg), 1, refkf=True)
tr.set_vocabulary(voc, 4)
tr.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
tr.set_history(3)
g = pkg.DeviceBuffer(640*480); d = pkg.DeviceBuffer(640*480*4)
for f in range(3):
    g.upload(frames[f][0]); d.upload(frames[f][1])
    tr.step_device(g.ptr, d.ptr)
    tr.synchronize()
    print(f, 'trk', tr.trk(), 'state', {k: v for k, v in tr.state().items() if k != 'Tcw'}, tr.status())
    w, v, n = tr.bow(0)
    print('  bow', len(w), (n >= 0).sum())
