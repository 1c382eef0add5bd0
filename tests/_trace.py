"""Per-decision trace records comparable between the oracle and the kernel's debug trace."""
import numpy as np

M64 = (1 << 64) - 1


def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sem_pack(owner, is_in, t0, t1):
    return (t0 & 0xFFFF) | ((t1 & 0xFFFF) << 16) | ((owner & 0xFF) << 32) | ((is_in & 1) << 40) | (1 << 41)


class PortMap:
    def __init__(self, cm):
        self.cm = cm
        self.sidx = {sid: i for i, sid in enumerate(cm.switch_ids)}
        self.pid = {}
        for s, pl in enumerate(cm.ports):
            for j, p in enumerate(pl):
                self.pid[p] = 4 * s + j
        self.kidx = {st: i for i, st in enumerate(cm.stations)}

    def checksum(self, sem):
        c = 0
        for p, rec in sem.items():
            r = sem_pack(rec[0], 1 if rec[1] == "in" else 0, int(rec[3]), int(rec[4]))
            c = (c + mix64((self.pid[p] << 42) ^ r)) & M64
        return c

    def state_of(self, obs):
        cm = self.cm
        s = self.sidx[(int(obs[0]), int(obs[1]))]
        P = len(cm.ports[s])
        sem, tgt, dl = obs[2:2 + P], obs[2 + P:2 + 3 * P], obs[2 + 3 * P:2 + 4 * P]
        slot = [i for i in range(P) if dl[i] != -1][0]
        k = self.kidx[(int(tgt[2 * slot]), int(tgt[2 * slot + 1]))]
        bits = sum(int(b) << j for j, b in enumerate(sem))
        return (bits * cm.K + k) * 3 + int(dl[slot])


def oracle_recorder(cm, out):
    pm = PortMap(cm)

    def hook(env, obs, action, reward, post):
        sw = pm.sidx[tuple(int(x) for x in obs[:2])]
        out.append((int(env.now()), sw, int(env.active_train), int(action), pm.state_of(obs), int(reward),
                    pm.checksum(env.sem), pm.sidx[tuple(post["next_switch"])]))
    return hook


def decode_kernel_trace(tr):
    res = []
    for w0, w1, w2, w3 in tr.astype(np.uint64).tolist():
        now = w0 & 0xFFFF
        now = now - 0x10000 if now >= 0x8000 else now
        rew = (w1 >> 32) & 0xFFFFFFFF
        rew = rew - (1 << 32) if rew >= (1 << 31) else rew
        res.append((now, (w0 >> 16) & 0xFFFF, (w0 >> 32) & 0xFFFF, (w0 >> 48) & 0xFFFF, w1 & 0xFFFFFFFF, rew, w2,
                    w3 & 0xFFFFFFFF))
    return res
