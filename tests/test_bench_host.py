"""Host logic of bench.py that needs no GPU: the untimed settle-step count, the pass kernel names."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_settle_steps_fill_the_warmup_to_settle_ms():
    # 5 warmup steps of 0.5 ms: 2.5 ms done, 27.5 ms more = 55 steps
    assert bench.settle_steps_needed(2.5e-3, 5, 30.0) == 55
    # a warmup that already lasted long enough adds nothing
    assert bench.settle_steps_needed(0.17, 2, 30.0) == 0
    # partial steps round up, so the warmup lasts at least settle_ms
    assert bench.settle_steps_needed(1.0e-3, 1, 2.5) == 2


def test_settle_steps_disabled_and_capped():
    assert bench.settle_steps_needed(1e-3, 3, 0.0) == 0
    assert bench.settle_steps_needed(1e-3, 0, 30.0) == 0
    # microsecond steps (C2 issued eagerly) stop at the cap
    assert bench.settle_steps_needed(3e-6, 3, 30.0) == 2000
    assert bench.settle_steps_needed(3e-6, 3, 30.0, cap=500) == 500


def test_stencil_kernel_names_follow_the_launch_rules():
    """The rocprof names the bench looks its pass up by: the 4096^2 x 2 pass (537 MB)
    streams its stores, a 10-deep pass of <= 192 MiB (C3's 1024^2 x 2) stores
    through the caches (vk_stencil_ps10.hip), variant 40 is the stage-split pass."""
    whole = 16 * 4096 * 4096 * 2
    assert bench.stencil_kernel_name(20, 10, 'fma', whole) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 0, 0>'
    assert bench.stencil_kernel_name(20, 10, 'fma', 16 * 1024 * 1024 * 2) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 2, 0>'
    assert bench.stencil_kernel_name(20, 9, 'fma', 16 * 1024 * 1024 * 2) == 'vk_ps::k_diffuse_ps<9, 4, 2, true, 0, 0>'
    assert bench.stencil_kernel_name(40, 10, 'fma', whole) == 'vk_sp::k_diffuse_sp<10, 4, 2, 5, true, 0>'
    assert bench.stencil_kernel_name(70, 10, 'fma', whole) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 0, 16>'
    assert bench.stencil_kernel_name(70, 10, 'fma', 16 * 1024 * 1024 * 2) == 'vk_ps::k_diffuse_ps<10, 4, 2, true, 2, 16>'
    assert bench.stencil_kernel_name(70, 9, 'fma', whole) == 'vk_ps::k_diffuse_ps<9, 4, 2, true, 0, 0>'
    assert bench.stencil_kernel_name(40, 9, 'fma', whole) == 'vk_ps::k_diffuse_ps<9, 4, 2, true, 0, 0>'
    assert bench.stencil_kernel_name(6, 9, 'exact') == 'vk_nt::k_diffuse_wl<9, 6, false>'
    assert bench.stencil_kernel_name(6, 10, 'exact') == 'vk_nt::k_diffuse_wl<10, 3, false>'
    # the tolerance mode's wave-tile FMA form is retired: variant 6 selects the pair-sum pass
    assert bench.stencil_kernel_name(6, 9, 'fma') == 'vk_ps::k_diffuse_ps<9, 4, 2, true, 0, 0>'
    assert bench.stencil_kernel_name(20, 13, 'fma') == 'vk_nt::k_diffuse_wl<13, 6, false>'.replace('vk_nt::', '')


class _FakeChild:
    def __init__(self, cmd, rc=0):
        self.cmd, self.rc, self.signals = cmd, rc, []

    def wait(self):
        return self.rc

    def send_signal(self, s):
        self.signals.append(s)


def test_gpus_n_starts_n_ranks_as_a_child_before_any_gpu_call():
    """--gpus N without a launcher: torch.distributed.run with N ranks, started as
    a child process (never an exec), whose exit code the parent returns; nothing
    before it initialised the GPU."""
    import torch
    started = []

    def popen(cmd):
        assert not torch.cuda.is_initialized()
        started.append(_FakeChild(cmd, rc=3))
        return started[-1]
    argv = ['--gpus', '4', '--steps', '5', '--warmup', '2', '--dist-backend', 'gloo']
    rc = bench.launch_ranks(argv, environ={}, popen=popen)
    assert rc == 3 and len(started) == 1
    cmd = started[0].cmd
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert int(cmd[cmd.index('--master-port') + 1]) > 0
    i = cmd.index(os.path.join(bench.REPO, 'bench.py'))
    assert cmd[i + 1:] == argv          # the ranks see the same arguments (and WORLD_SIZE = 4)
    assert not torch.cuda.is_initialized()


def test_gpus_flag_inside_a_launcher_or_on_one_gpu_runs_in_process():
    never = lambda cmd: (_ for _ in ()).throw(AssertionError('no child expected'))
    assert bench.launch_ranks(['--gpus', '8'], environ={'WORLD_SIZE': '8'}, popen=never) is None
    assert bench.launch_ranks([], environ={}, popen=never) is None
    assert bench.launch_ranks(['--gpus', '1'], environ={}, popen=never) is None
    assert bench.launch_ranks(['--gpus=2'], environ={'WORLD_SIZE': '2'}, popen=never) is None


def test_gpus_flag_mismatching_the_launcher_exits_nonzero():
    import pytest
    never = lambda cmd: (_ for _ in ()).throw(AssertionError('no child expected'))
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks(['--gpus', '8'], environ={'WORLD_SIZE': '2'}, popen=never)
    assert e.value.code not in (0, None)
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks(['--gpus', '0'], environ={}, popen=never)
    assert e.value.code not in (0, None)


def test_bench_script_with_wrong_world_size_fails_before_importing_lens_amd():
    """The real entry point: a mismatch exits non-zero with the message, and the
    check runs before lens_amd (and its HIP library) is imported."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE='2')
    p = subprocess.run([sys.executable, '-X', 'importtime', os.path.join(bench.REPO, 'bench.py'), '--gpus', '4'],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert 'WORLD_SIZE=2' in p.stderr
    assert 'lens_amd' not in p.stderr.replace('WORLD_SIZE', '')



def test_stencil_settings_pick_the_split_pass_for_row_bands():
    """One GPU: the line-aligned pair-sum pass (variant 70) on 64-row tiles; row bands
    at N > 4 and C3: the stage-split 10-deep pass (variant 40) with auto chunk rows; N =
    2 / 4: variant 20; an explicit --stencil-kernel wins; the exact mode never takes the
    split pass."""
    args = bench.parse([])
    assert bench.stencil_settings(args, 1) == ('fma', 10, 70, 64)
    assert bench.stencil_settings(bench.parse(['--stencil-kernel', '20']), 1) == ('fma', 10, 20, 64)
    args = bench.parse([])
    assert bench.stencil_settings(args, 8) == ('fma', 10, 40, 0)
    assert bench.stencil_settings(args, 4) == ('fma', 10, 20, 0)
    assert bench.stencil_settings(args, 2) == ('fma', 10, 20, 0)
    args = bench.parse(['--stencil-kernel', '20'])
    assert bench.stencil_settings(args, 8) == ('fma', 10, 20, 0)
    args = bench.parse(['--stencil-kernel', '40'])
    assert bench.stencil_settings(args, 4) == ('fma', 10, 40, 0)
    args = bench.parse(['--stencil-mode', 'exact'])
    assert bench.stencil_settings(args, 2)[2] == 20
    # C3 (1024^2) on one GPU: 10-deep split passes, auto rows; its exact mode keeps depth 9
    assert bench.stencil_settings(bench.parse(['--workload', 'c3']), 1) == ('fma', 10, 40, 0)
    assert bench.stencil_settings(bench.parse(['--workload', 'c3', '--stencil-mode', 'exact']), 1) == \
        ('exact', 9, 20, 0)
    assert bench.stencil_kernel_name(40, 10, 'fma') == 'vk_sp::k_diffuse_sp<10, 4, 2, 5, true, 0>'


def test_pass_plan_restates_the_library_planner():
    """bench.pass_plan (the passes time_stencil_pass divides a step's time by)
    follows vk_diffuse: 10-deep blocks for multiples of 10, else odd passes of at
    most 9 (depth 10's fallback) or the odd depth, as many as the parity needs."""
    assert bench.pass_plan(100, 10) == [10] * 10
    for n_sub, depth in ((100, 9), (501, 9), (1001, 11), (37, 10), (100, 7), (3, 15)):
        ks = bench.pass_plan(n_sub, depth)
        d = min(9 if depth == 10 else depth | 1, 15)
        assert sum(ks) == n_sub and all(k % 2 == 1 and k <= d for k in ks), (n_sub, depth, ks)
        assert len(ks) % 2 == n_sub % 2
