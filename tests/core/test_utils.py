"""Unit tests of ``zookeeper_amd.core.utils`` / ``core.typecheck`` (the
reference's ``zookeeper/core/utils_test.py`` and ``zookeeper/test_version.py``
cover the predicates and the version string; the extra cases pin the
naming, CLI-value parsing, immutability and type-checking helpers that the
rest of the config system relies on)."""

from typing import Annotated, Any, Callable, Dict, List, Optional, Sequence, Tuple, Type, Union

import pytest

import zookeeper_amd
from zookeeper_amd.core import utils
from zookeeper_amd.core.component import component
from zookeeper_amd.core.factory import factory
from zookeeper_amd.core.typecheck import check_type


def test_version_is_a_string():
    assert isinstance(zookeeper_amd.__version__, str) and zookeeper_amd.__version__


def test_is_component_class():
    assert not utils.is_component_class(5)
    assert not utils.is_component_class(lambda: "foo")

    class Plain:
        pass

    assert not utils.is_component_class(Plain)

    @component
    class Comp:
        pass

    assert utils.is_component_class(Comp)
    assert not utils.is_component_class(Comp())

    class Undecorated(Comp):
        pass

    # only decorated classes are components, not their plain subclasses
    assert not utils.is_component_class(Undecorated)


def test_is_component_instance():
    assert not utils.is_component_instance(5)

    @component
    class Comp:
        pass

    assert not utils.is_component_instance(Comp)
    assert utils.is_component_instance(Comp())


def test_is_factory_class_and_instance():
    class NotFactory:
        def build(self) -> object:
            pass

    assert not utils.is_factory_class(NotFactory)
    assert not utils.is_factory_instance(NotFactory())

    @factory
    class Fac:
        def build(self) -> object:
            pass

    assert utils.is_factory_class(Fac)
    assert not utils.is_factory_class(Fac())
    assert utils.is_factory_instance(Fac())
    assert not utils.is_factory_instance(Fac)


@pytest.mark.parametrize("name", ["FooBar", "fooBar", "Foo_Bar", "foo_bar"])
def test_convert_to_snake_case(name):
    assert utils.convert_to_snake_case(name) == "foo_bar"


@pytest.mark.parametrize("raw,value", [
    ("5", 5), ("1e-3", 1e-3), ("[1, 2.5]", [1, 2.5]), ("(3, 4)", (3, 4)),
    ("{'x': 'y'}", {"x": "y"}), ("None", None), ("True", True), ("False", False),
    ("hello", "hello"), ("https://a/b@c", "https://a/b@c"), ("'quoted'", "quoted")])
def test_parse_value_from_string(raw, value):
    assert utils.parse_value_from_string(raw) == value


def test_is_immutable():
    for v in (None, 1, 1.5, True, "s", frozenset({1}), (1, "a", None), ()):
        assert utils.is_immutable(v), v
    for v in ([1], {"a": 1}, {1}, (1, [2]), ((1,),), object()):
        assert not utils.is_immutable(v), v
    f = utils.wrap_in_callable([1, 2])
    assert f() == [1, 2] and f() is f()


def test_generate_subclasses_and_component_subclasses():
    @component
    class Base:
        pass

    class Mid(Base):
        pass

    @component
    class Leaf(Mid):
        pass

    assert list(utils.generate_subclasses(Base)) == [Base, Mid, Leaf]
    assert list(utils.generate_component_subclasses(Base)) == [Base, Leaf]


def test_ancestors_with_field_closest_first():
    from zookeeper_amd import ComponentField, Field, configure

    @component
    class Child:
        x: int = Field()

    @component
    class Middle:
        x: int = Field(1)
        child: Child = ComponentField(Child)

    @component
    class Root:
        x: int = Field(2)
        middle: Middle = ComponentField(Middle)

    r = Root()
    configure(r, {})
    anc = list(utils.generate_component_ancestors_with_field(r.middle.child, "x"))
    assert anc == [r.middle, r]
    assert r.middle.child.x == 1


@pytest.mark.parametrize("value,tp,ok", [
    (1, int, True), (1, float, True), (1.0, int, False), (True, int, True),
    (None, Optional[int], True), ("a", Optional[int], False),
    ([1, 2], List[int], True), ([1, "2"], List[int], False),
    ((1, "a"), Tuple[int, str], True), ((1, 2, 3), Tuple[int, ...], True),
    ((1,), Tuple[int, str], False), ({"a": 1}, Dict[str, int], True),
    ({"a": "b"}, Dict[str, int], False), (1, Union[str, int], True),
    (int, Type[int], True), (bool, Type[int], True), (str, Type[int], False),
    (len, Callable[..., int], True), (3, Callable, False), ([1.0], Sequence[float], True),
    ("x", Any, True), (object(), object, True),
    # plain-class fast path and memoised / unhashable typing annotations
    (1, complex, True), (2.5, complex, True), (None, type(None), True), (0, type(None), False),
    ((1, 2), Tuple[int, int], True), ((1, 2), Tuple[int, int], True),
    (1, Annotated[int, []], True), ("1", Annotated[int, []], False)])
def test_check_type(value, tp, ok):
    assert check_type(value, tp) is ok


def test_type_check_of_factory_uses_build_annotation():
    class Product:
        pass

    @factory
    class MakeProduct:
        def build(self) -> Product:
            return Product()

    assert utils.type_check(MakeProduct(), Product)
    assert not utils.type_check(MakeProduct(), int)


def test_warn_prints_to_stderr(capsys):
    utils.warn("careful")
    assert capsys.readouterr().err.strip() == "WARNING: careful"
