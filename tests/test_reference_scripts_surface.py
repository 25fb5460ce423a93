"""The reference's entry scripts resolve against this package.

Reads ``/root/reference/legged_gym/scripts/{train,play}.py`` AS TEXT (``ast``; nothing of
the reference is imported or executed) and checks that every name they import and every
``env.`` / ``ppo_runner.`` / ``env_cfg.`` / ``train_cfg.`` / ``args.`` / ``task_registry.``
attribute path they use exists on the build's package, configs and classes.  It runs in
the build container only: ``/root/reference`` does not exist on the GPU box (skipped there).
"""
import ast
import importlib
import inspect
import os

import pytest

REF = "/root/reference/legged_gym/scripts"
SCRIPTS = ("train.py", "play.py")
ROOTS = ("env", "ppo_runner", "env_cfg", "train_cfg", "args", "task_registry")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference scripts are only in the build container")


def _tree(name):
    with open(os.path.join(REF, name)) as f:
        return ast.parse(f.read())


def _imports(tree):
    """[(module, name or None)] of every import statement."""
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            out += [(a.name, None) for a in node.names]
        elif isinstance(node, ast.ImportFrom):
            out += [(node.module, a.name) for a in node.names]
    return out


def _chains(tree):
    """Attribute chains rooted at one of ROOTS: ('env', 'max_episode_length'), ..."""
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Attribute) and not isinstance(getattr(node, "_parent", None), ast.Attribute):
            parts, cur = [], node
            while isinstance(cur, ast.Attribute):
                parts.append(cur.attr)
                cur = cur.value
            if isinstance(cur, ast.Name) and cur.id in ROOTS:
                out.add((cur.id,) + tuple(reversed(parts)))
    # keep only maximal chains (a.b.c implies a.b)
    return {c for c in out if not any(o != c and o[:len(c)] == c for o in out)} | out


def _instance_attrs(cls):
    """Names a class and its bases define, or assign as ``self.<name>`` in any method."""
    names = set(dir(cls))
    for k in cls.__mro__:
        try:
            src = inspect.getsource(k)
        except (OSError, TypeError):
            continue
        for node in ast.walk(ast.parse(src.lstrip() if src[:1].isspace() else src)):
            targets = []
            if isinstance(node, ast.Assign):
                targets = node.targets
            elif isinstance(node, (ast.AnnAssign, ast.AugAssign)):
                targets = [node.target]
            for t in targets:
                for e in (t.elts if isinstance(t, ast.Tuple) else [t]):
                    if isinstance(e, ast.Attribute) and isinstance(e.value, ast.Name) and e.value.id == "self":
                        names.add(e.attr)
    return names


def test_reference_script_imports_resolve():
    import isaacgym  # noqa: F401
    for script in SCRIPTS:
        for mod, name in _imports(_tree(script)):
            m = importlib.import_module(mod)
            if name not in (None, "*"):
                assert hasattr(m, name), f"{script}: from {mod} import {name} fails on the build"


def test_reference_script_attribute_paths_resolve():
    import isaacgym  # noqa: F401
    import legged_gym.envs  # noqa: F401
    from legged_gym.envs.base.legged_robot import LeggedRobot
    from legged_gym.envs.base.humanoid import HumanoidRobot
    from legged_gym.utils import get_args, task_registry
    from rsl_rl.algorithms import PPO
    from rsl_rl.runners import OnPolicyRunner
    chains = set()
    for script in SCRIPTS:
        chains |= _chains(_tree(script))
    assert chains, "no attribute paths found"
    args = get_args([])
    env_attrs = _instance_attrs(LeggedRobot) | _instance_attrs(HumanoidRobot)
    runner_attrs, alg_attrs = _instance_attrs(OnPolicyRunner), _instance_attrs(PPO)
    for task in ("go2", "g1", "h1", "h1_2"):
        env_cfg, train_cfg = task_registry.get_cfgs(task)
        objs = {"env_cfg": env_cfg, "train_cfg": train_cfg, "args": args, "task_registry": task_registry}
        for chain in sorted(chains):
            root, path = chain[0], chain[1:]
            if root in objs:
                o = objs[root]
                for i, a in enumerate(path):
                    assert hasattr(o, a), f"{task}: {'.'.join(chain[:i + 2])} does not resolve"
                    o = getattr(o, a)
            elif root == "env":
                assert path[0] in env_attrs, f"env.{path[0]} is not an attribute of the build's LeggedRobot"
                if path[0] == "cfg" and len(path) > 1:
                    o = env_cfg
                    for a in path[1:]:
                        assert hasattr(o, a), f"{task}: env.{'.'.join(path)} does not resolve"
                        o = getattr(o, a)
            elif root == "ppo_runner":
                assert path[0] in runner_attrs, f"ppo_runner.{path[0]} is not an OnPolicyRunner attribute"
                if path[0] == "alg" and len(path) > 1:
                    assert path[1] in alg_attrs, f"ppo_runner.alg.{path[1]} is not a PPO attribute"


def test_build_scripts_import_what_the_reference_scripts_import():
    """The build's train.py / play.py import the same names from the same modules."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "unitree-rl-gym_amd", "legged_gym",
                        "scripts")
    for script in SCRIPTS:
        with open(os.path.join(here, script)) as f:
            mine = {(m, n) for m, n in _imports(ast.parse(f.read())) if m and m.startswith(("legged_gym", "isaacgym"))}
        ref = {(m, n) for m, n in _imports(_tree(script)) if m and m.startswith(("legged_gym", "isaacgym"))}
        assert ref <= mine, f"{script}: the build's script lacks {sorted(ref - mine)}"
