"""Parity tests for ``@factory``, ``@task``, the CLI and the helper predicates
(reference: zookeeper/core/{factory,task,cli,utils}_test.py, zookeeper/test_version.py).

click 8.4 removed ``CliRunner(mix_stderr=...)``; stdout is read from
``result.stdout`` here.
"""

import pytest
from click.testing import CliRunner

import zookeeper_amd
from zookeeper_amd import ComponentField, Field, component, factory, task
from zookeeper_amd.core import utils
from zookeeper_amd.core.factory import FACTORY_REGISTRY

# --------------------------------------------------------------------------- #
# @factory
# --------------------------------------------------------------------------- #

BUILD_MSG = (
    r"Classes decorated with @factory must implement a `build\(\)` method taking "
    "precisely one positional argument"
)


def test_factory_requires_build():
    with pytest.raises(TypeError, match=BUILD_MSG):

        @factory
        class NoBuild:
            pass


@pytest.mark.parametrize("src", ["def build(self, a, b): pass", "def build(this): pass"])
def test_factory_build_signature(src):
    ns = {}
    exec(src, ns)
    cls = type("Bad", (), {"build": ns["build"]})
    with pytest.raises(TypeError, match=BUILD_MSG):
        factory(cls)


def test_factory_requires_return_annotation():
    with pytest.raises(
        TypeError,
        match=r"The `build\(\)` method of a @factory class must have an annotated return type",
    ):

        @factory
        class NoAnnotation:
            def build(self):
                pass


def test_factory_registered_by_return_type():
    class Product:
        pass

    @factory
    class Maker:
        def build(self) -> Product:
            return Product()

    assert Maker in FACTORY_REGISTRY.get(Product, set())


def test_factory_build_result_is_type_checked_and_cached():
    @factory
    class Liar:
        def build(self) -> int:
            return "not an int"

    with pytest.raises(TypeError, match="which is not satisfied by the return value"):
        Liar().build()

    @factory
    class Once:
        def build(self) -> list:
            return []

    o = Once()
    assert o.build() is o.build()


def test_unconfigured_factory_strings():
    @factory
    class Maker:
        x: int = Field(1)

        def build(self) -> int:
            return self.x

    m = Maker()
    assert str(m) == "<Unconfigured factory 'Maker' instance>"
    assert repr(m) == "<Unconfigured factory 'Maker' instance>"


# --------------------------------------------------------------------------- #
# @task
# --------------------------------------------------------------------------- #


def test_tasks_accept_argumentless_run_variants(clean_cli):
    @task
    class Plain:
        def run(self):
            pass

    @task
    class Klass:
        @classmethod
        def run(cls):
            pass

    @task
    class Static:
        @staticmethod
        def run():
            pass


def test_task_requires_run(clean_cli):
    with pytest.raises(TypeError, match="Classes decorated with @task must define a `run` method."):

        @task
        class NoRun:
            pass


def test_task_run_with_args(clean_cli):
    with pytest.raises(
        TypeError,
        match=r"^A @task class must define a `run` method taking no arguments except `self`",
    ):

        @task
        class Bad:
            def run(a, b):
                pass


def test_task_name_conflict(clean_cli):
    @task
    class FooBar:
        def run(self):
            pass

    with pytest.raises(ValueError, match="Task naming conflict"):

        @task
        class foo_bar:  # noqa: N801 - same snake-case name on purpose
            def run(self):
                pass


# --------------------------------------------------------------------------- #
# CLI
# --------------------------------------------------------------------------- #


@pytest.fixture
def echo_task(clean_cli):
    @task
    class EchoTask:
        a: int = Field()
        b: str = Field("foo")
        c: bool = Field(False)

        def run(self):
            print(self.a, self.b, self.c)

    return clean_cli, CliRunner()


@pytest.mark.parametrize("name", ["echo_task", "EchoTask", "Echo_Task", "echoTask"])
def test_command_aliases(echo_task, name):
    cli, runner = echo_task
    assert runner.invoke(cli, [name, "a=5"]).exit_code == 0


def test_unknown_command(echo_task):
    cli, runner = echo_task
    assert runner.invoke(cli, ["NotEchoTask", "a=5"]).exit_code != 0


@pytest.mark.parametrize(
    "args,expected",
    [
        (["a=5"], "5 foo False\n"),
        (["a=5", "b=bar", "c=True"], "5 bar True\n"),
        (["a=5", "b=https://some-path/foo/bar@somewhere"], "5 https://some-path/foo/bar@somewhere False\n"),
        (["a=5", "--c"], "5 foo True\n"),
        (["a=5", "--no-c"], "5 foo False\n"),
        (["a=1", "a=2"], "2 foo False\n"),  # later duplicates win
    ],
)
def test_cli_values(echo_task, args, expected):
    cli, runner = echo_task
    result = runner.invoke(cli, ["echo_task", *args])
    assert result.exit_code == 0, result.output
    assert result.stdout == expected


@pytest.mark.parametrize("bad", ["x-y=1.0", "x@y=1.0", "a=b=c", "novalue"])
def test_cli_rejects_malformed_tokens(echo_task, bad):
    cli, runner = echo_task
    assert runner.invoke(cli, ["echo_task", "a=5", bad]).exit_code == 2


def test_cli_type_error_exits_1(echo_task):
    cli, runner = echo_task
    result = runner.invoke(cli, ["echo_task", "a=1.5"])
    assert result.exit_code == 1
    assert isinstance(result.exception, TypeError)


def test_cli_nested_keys(clean_cli):
    @component
    class Kid:
        x_Y_z: float = Field(0.0)

    @task
    class ParentTask:
        a: int = Field(2)
        kid: Kid = ComponentField(Kid)

        def run(self):
            print(self.a, self.kid.x_Y_z)

    result = CliRunner().invoke(clean_cli, ["ParentTask", "a=5", "kid.x_Y_z=1.0"])
    assert result.exit_code == 0
    assert result.stdout == "5 1.0\n"


def test_cli_component_and_factory_selection(clean_cli):
    class Base:
        name = "abstract"

    @component
    class BaseComponent(Base):
        name = "component"

    @factory
    class BaseFactory:
        def build(self) -> Base:
            value = Base()
            value.name = "factory"
            return value

    @task
    class PickBase:
        base: Base = ComponentField()

        def run(self):
            print(self.base.name)

    runner = CliRunner()
    assert runner.invoke(clean_cli, ["pick_base"]).exit_code == 1
    result = runner.invoke(clean_cli, ["pick_base", "base=BaseComponent"])
    assert (result.exit_code, result.stdout) == (0, "component\n")
    result = runner.invoke(clean_cli, ["pick_base", "base=BaseFactory"])
    assert (result.exit_code, result.stdout) == (0, "factory\n")


# --------------------------------------------------------------------------- #
# utils
# --------------------------------------------------------------------------- #


def test_component_predicates():
    class Plain:
        def build(self) -> object:
            pass

    @component
    class Comp:
        pass

    @factory
    class Fact:
        def build(self) -> object:
            pass

    for not_component in (5, lambda: "foo", Plain, Plain(), Comp()):
        assert not utils.is_component_class(not_component)
    assert utils.is_component_class(Comp) and utils.is_component_class(Fact)
    assert utils.is_component_instance(Comp()) and not utils.is_component_instance(Comp)
    assert utils.is_factory_class(Fact) and not utils.is_factory_class(Comp)
    assert not utils.is_factory_class(Plain) and not utils.is_factory_class(Fact())
    assert utils.is_factory_instance(Fact()) and not utils.is_factory_instance(Fact)
    assert not utils.is_factory_instance(Plain())


@pytest.mark.parametrize(
    "raw,value",
    [("5", 5), ("1e-3", 1e-3), ("[1,2.5]", [1, 2.5]), ("(3,4)", (3, 4)), ("{'x':'y'}", {"x": "y"}),
     ("None", None), ("True", True), ("hello", "hello"), ("https://a/b@c", "https://a/b@c")],
)
def test_parse_value_from_string(raw, value):
    assert utils.parse_value_from_string(raw) == value


@pytest.mark.parametrize("name", ["FooBar", "fooBar", "Foo_Bar", "foo_bar", "foo__bar"])
def test_snake_case(name):
    assert utils.convert_to_snake_case(name) == "foo_bar"


def test_is_immutable():
    for v in (None, 1, 1.0, True, "s", frozenset([1]), (1, "a", None)):
        assert utils.is_immutable(v)
    for v in ([], {}, (1, [2]), object()):
        assert not utils.is_immutable(v)


def test_version():
    assert hasattr(zookeeper_amd, "__version__") and "." in zookeeper_amd.__version__
