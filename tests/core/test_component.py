"""Behavioural parity tests for ``@component`` / ``configure``.

Each test pins one behaviour of the reference (zookeeper/core/component.py)
and cites the reference test that covers the same behaviour
(zookeeper/core/component_test.py).  Classes are defined inside the tests so
every test sees fresh classes.
"""

import abc
from typing import List, Tuple
from unittest import mock

import click
import pytest

from zookeeper_amd import ComponentField, Field, component, configure, factory
from zookeeper_amd.core.component import base_getattr


def make_pair():
    @component
    class Pair:
        left: int = Field()
        right: str = Field("foo")

    return Pair


# --- decorator validation (component_test.py:23-67) ----------------------- #


def test_rejects_functions():
    with pytest.raises(TypeError, match="Only classes can be decorated with @component."):
        component(lambda: None)


def test_rejects_abstract_classes():
    class Base(abc.ABC):
        @abc.abstractmethod
        def go(self):
            ...

    with pytest.raises(TypeError, match="Abstract classes cannot be decorated with @component."):
        component(Base)


def test_rejects_custom_init():
    class WithInit:
        def __init__(self, x):
            self.x = x

    with pytest.raises(
        TypeError, match="Component classes must not define a custom `__init__` method."
    ):
        component(WithInit)


def test_rejects_double_decoration():
    Pair = make_pair()
    with pytest.raises(TypeError, match="is already a component"):
        component(Pair)


# --- __init__ contract (component_test.py:70-100) -------------------------- #


def test_init_kwargs_set_fields():
    Pair = make_pair()
    p = Pair(left=2)
    assert (p.left, p.right) == (2, "foo")
    p = Pair(left=0, right="bar")
    assert (p.left, p.right) == (0, "bar")


def test_init_rejects_positional_and_unknown():
    Pair = make_pair()
    with pytest.raises(TypeError, match=r"takes 1 positional argument but 2 were given"):
        Pair("x")
    with pytest.raises(
        TypeError,
        match="Keyword arguments passed to component `__init__` must correspond to "
        "component fields. Received non-matching argument 'nope'",
    ):
        Pair(nope=0)


# --- configure: overrides and scoping (component_test.py:103-156) ---------- #


def test_configure_overrides_defaults():
    p = make_pair()()
    configure(p, {"left": 0, "right": "bar"})
    assert (p.left, p.right) == (0, "bar")


def test_scoped_configuration():
    @component
    class Leaf:
        n: int = Field()
        s: str = Field()
        v: List[float] = Field()

    @component
    class Mid:
        s: str = Field("mid")
        leaf: Leaf = ComponentField(Leaf)

    @component
    class Root:
        n: int = Field()
        s: str = Field()
        mid: Mid = ComponentField(Mid)

    r = Root()
    configure(
        r,
        {"n": 10, "mid.leaf.n": 15, "s": "root", "mid.leaf.s": "leaf", "mid.leaf.v": [0, 4.2]},
    )
    assert r.n == 10 and r.mid.leaf.n == 15
    # `s` configured at the root reaches `mid` (overriding its default), but the
    # leaf has its own scoped value.
    assert (r.s, r.mid.s, r.mid.leaf.s) == ("root", "root", "leaf")
    assert r.mid.leaf.v == [0, 4.2]


def test_module_docstring_example_precedence():
    """The scoping example of zookeeper/core/component.py:23-77."""

    @component
    class A:
        w: int = Field(3)
        x: int = Field()
        y: str = Field("foo")
        z: float = Field()

    @component
    class B:
        a: A = ComponentField(A)
        w: int = Field(5)
        x: int = Field()
        y: str = Field("bar")

    @component
    class C:
        b: B = ComponentField(B)
        x: int = Field()
        z: float = Field(3.14)

    c = C()
    configure(c, {"x": 5, "b.x": 10, "b.a.x": 15, "b.y": "baz", "b.a.z": 2.71})
    assert (c.b.a.w, c.b.a.x, c.b.a.y, c.b.a.z) == (3, 15, "baz", 2.71)
    assert (c.b.w, c.b.x, c.b.y) == (5, 10, "baz")
    assert (c.x, c.z) == (5, 3.14)


def test_parent_configured_value_beats_child_default_but_init_kwarg_does_not():
    @component
    class Kid:
        v: int = Field(1)

    @component
    class Dad:
        v: int = Field(2)
        kid: Kid = ComponentField(Kid)

    d = Dad()
    configure(d, {"v": 9})
    assert d.kid.v == 9

    d = Dad(v=3)
    configure(d, {})
    assert d.v == 3 and d.kid.v == 1


def test_configure_does_not_mutate_callers_dict():
    p = make_pair()()
    conf = {"left": 1}
    configure(p, conf)
    assert conf == {"left": 1}


# --- auto-instantiation (component_test.py:159-191) ------------------------ #


def test_single_candidate_is_instantiated_with_warning(capsys):
    class Shape:
        pass

    @component
    class Square(Shape):
        pass

    @component
    class Holder:
        shape: Shape = ComponentField()

    capsys.readouterr()
    h = Holder()
    configure(h, {})
    assert isinstance(h.shape, Square)
    assert "is the only concrete component class" in capsys.readouterr().err

    @component
    class Circle(Shape):
        pass

    with pytest.raises(
        ValueError,
        match=r"^Component field 'Holder.shape' of type 'Shape' has no default or configured class.",
    ):
        configure(Holder(), {})


# --- missing values / interactive (component_test.py:194-279) -------------- #


def test_missing_value_error_uses_given_name():
    with pytest.raises(
        ValueError,
        match=r"^No configuration value found for annotated field 'NAMED.left' of type 'int'.",
    ):
        configure(make_pair()(), {"right": "bar"}, name="NAMED")


def test_interactive_prompts_for_missing_value():
    p = make_pair()()
    with mock.patch("click.prompt", return_value=42) as prompt:
        configure(p, {"right": "bar"}, interactive=True)
    assert (p.left, p.right) == (42, "bar")
    prompt.assert_called_once()


def test_interactive_prompts_for_subclass_in_sorted_order():
    class Animal:
        pass

    @component
    class Cat(Animal):
        pass

    @component
    class Ant(Animal):
        pass

    class Bird(Animal):  # not a component: excluded from the menu
        pass

    @component
    class BirdB(Bird):
        pass

    @component
    class BirdA(Bird):
        pass

    @component
    class Zoo:
        animal: Animal = ComponentField()

    for index, expected in enumerate([Ant, BirdA, BirdB, Cat]):
        z = Zoo()
        with mock.patch("click.prompt", return_value=index) as prompt:
            configure(z, {}, interactive=True)
        assert type(z.animal) is expected
        prompt.assert_called_once()


# --- str / repr golden strings (component_test.py:282-331) ----------------- #


def test_str_and_repr_golden():
    @component
    class One:
        a: int = Field()

    @component
    class Two:
        a: int = Field()
        b: str = Field()
        c: List[float] = Field()
        d: int = Field(allow_missing=True)
        one: One = ComponentField()

    @component
    class Top:
        b: str = Field("bar")
        one: One = ComponentField(One)
        two: Two = ComponentField(Two)

    t = Top()
    assert repr(t) == "<Unconfigured component 'Top' instance>"
    configure(t, {"one.a": 5, "two.a": 10, "b": "foo", "two.c": [1.5, -1.2]}, name="top")
    assert click.unstyle(repr(t)) == (
        'Top(b="foo", one=One(a=5), two=Two(a=10, b=<inherited value>, c=[1.5, -1.2], '
        "d=<missing>, one=<inherited component instance>))"
    )
    assert click.unstyle(str(t)) == "\n".join(
        [
            "Top(",
            '    b="foo",',
            "    one=One(",
            "        a=5",
            "    ),",
            "    two=Two(",
            "        a=10,",
            "        b=<inherited value>,",
            "        c=[1.5, -1.2],",
            "        d=<missing>,",
            "        one=<inherited component instance>",
            "    )",
            ")",
        ]
    )


def test_callable_values_print_as_placeholder():
    @component
    class WithFn:
        fn: object = Field(lambda: len)

    w = WithFn()
    configure(w, {})
    assert repr(w) == "WithFn(fn=<callable>)"


# --- type checking (component_test.py:334-346) ----------------------------- #


def test_plain_fields_are_type_checked_lazily():
    p = make_pair()()
    configure(p, {"left": 4.5}, name="x")  # no error yet
    with pytest.raises(
        TypeError,
        match="Field 'left' of component 'x' is annotated with type '<class 'int'>', "
        "which is not satisfied by value 4.5.",
    ):
        p.left


def test_int_satisfies_float():
    @component
    class F:
        x: float = Field()

    f = F()
    configure(f, {"x": 3})
    assert f.x == 3


# --- subclass re-defaulting (component_test.py:349-358) -------------------- #


def test_overriding_a_field_with_a_plain_value_is_an_error():
    @component
    class Super:
        foo: str = Field("bar")

    with pytest.raises(ValueError, match="Field 'foo' is defined on super-class"):

        @component
        class Sub(Super):
            foo = 1


def test_subclass_can_redefault_without_annotation():
    @component
    class Super:
        foo: str = Field("bar")

    @component
    class Sub(Super):
        foo = Field("baz")

    s = Sub()
    configure(s, {})
    assert s.foo == "baz"
    assert Sub.__component_fields__["foo"].type is str


# --- factories as field values (component_test.py:361-461) ----------------- #


def test_factory_return_type_checks(capsys):
    class Base:
        pass

    class Impl(Base):
        pass

    @factory
    class MakesBase:
        def build(self) -> Base:
            return Impl()

    @factory
    class MakesImpl:
        def build(self) -> Impl:
            return Impl()

    @factory
    class MakesTriple:
        def build(self) -> Tuple[int, int, int]:
            return (1, 2, 3)

    @component
    class UsesBase:
        base: Base = ComponentField(MakesBase)

    @component
    class UsesImpl:
        base: Base = ComponentField(MakesImpl)

    @component
    class UsesTriple:
        base: Tuple[float, float, float] = ComponentField(MakesTriple)

    assert isinstance(UsesBase().base, Impl)
    assert isinstance(UsesImpl().base, Impl)
    capsys.readouterr()
    assert UsesTriple().base == (1, 2, 3)
    assert capsys.readouterr().err == (
        "WARNING: Unable to check that typing.Tuple[int, int, int] is a sub-type of "
        "typing.Tuple[float, float, float].\n"
    )


def test_factory_builds_once_and_base_getattr_sees_factory():
    calls = []

    @factory
    class Counter:
        start: int = Field(0)

        def build(self) -> list:
            calls.append(1)
            return [self.start]

    @component
    class Holder:
        counter: list = ComponentField(Counter)

    h = Holder()
    configure(h, {"counter.start": 4})
    assert h.counter == [4]
    assert h.counter is h.counter
    assert len(calls) == 1
    assert isinstance(base_getattr(h, "counter"), Counter)
    assert "Counter(start=4)" in repr(h)


def test_value_inherited_through_a_factory_parent():
    @component
    class Kid:
        x: int = Field()

    @factory
    class Maker:
        kid: Kid = ComponentField(Kid)
        x: int = Field(5)

        def build(self) -> int:
            return self.kid.x

    m = Maker()
    configure(m, {})
    assert m.kid.x == 5 and m.build() == 5


def test_inherited_factory_value():
    @factory
    class Five:
        def build(self) -> int:
            return 5

    @component
    class Kid:
        x: int = ComponentField()

    @component
    class Dad:
        kid: Kid = ComponentField(Kid)
        x: int = ComponentField(Five)

    d = Dad()
    configure(d, {})
    assert (d.x, d.kid.x) == (5, 5)

    d = Dad()
    configure(d, {"kid.x": 7})
    assert (d.x, d.kid.x) == (5, 7)


def test_unmatched_class_name_fails_type_check_during_configure():
    class Base:
        pass

    @component
    class Impl(Base):
        pass

    @component
    class Holder:
        thing: Base = ComponentField()

    with pytest.raises(TypeError, match="which is not satisfied by value 'NoSuchClass'"):
        configure(Holder(), {"thing": "NoSuchClass"})


@pytest.mark.parametrize("spelling", ["FooBarImpl", "foo_bar_impl", "fooBarImpl"])
def test_component_field_resolves_class_names(spelling):
    class Base:
        pass

    @component
    class FooBarImpl(Base):
        pass

    @component
    class Other(Base):
        pass

    @component
    class Holder:
        thing: Base = ComponentField()

    h = Holder()
    configure(h, {"thing": spelling})
    assert isinstance(h.thing, FooBarImpl)


# --- post-configure hooks (component_test.py:464-499) ---------------------- #


def test_post_configure_validation_and_call_order():
    with pytest.raises(
        TypeError,
        match="The `__post_configure__` attribute of a @component class must be a method.",
    ):

        @component
        class Bad1:
            __post_configure__ = 3.14

    with pytest.raises(
        TypeError,
        match="The `__post_configure__` method of a @component class must take no "
        "arguments except `self`",
    ):

        @component
        class Bad2:
            def __post_configure__(self, x):
                pass

    order = []

    @component
    class Kid:
        a: int = Field(0)

        def __post_configure__(self):
            order.append("kid")

    @component
    class Dad:
        a: int = Field(0)
        b: float = Field(3.14)
        kid: Kid = ComponentField(Kid)

        def __post_configure__(self):
            order.append("dad")
            self.total = self.a + self.b

    d = Dad()
    configure(d, {"a": 1, "b": -3.14})
    assert d.total == 1 - 3.14
    assert order == ["kid", "dad"]


# --- key validation (component_test.py:502-541) ---------------------------- #


def test_unknown_keys_are_rejected_with_scoped_names():
    @component
    class Kid:
        a: int = Field(1)

    @component
    class Dad:
        b: str = Field("foo")
        kid: Kid = ComponentField(Kid)

    @component
    class Grandpa:
        c: float = Field(3.14)
        dad: Dad = ComponentField(Dad)

    with pytest.raises(
        ValueError, match="Key 'd' does not correspond to any field of component 'Grandpa'."
    ):
        configure(Grandpa(), {"d": "bar"})
    # `b` lives on the child: it must be qualified.
    with pytest.raises(
        ValueError, match="Key 'b' does not correspond to any field of component 'Grandpa'."
    ):
        configure(Grandpa(), {"b": "bar"})
    g = Grandpa()
    configure(g, {"dad.b": "bar"})
    assert g.dad.b == "bar"
    with pytest.raises(
        ValueError,
        match="Key 'zzz' does not correspond to any field of component 'Grandpa.dad'.",
    ):
        configure(Grandpa(), {"dad.zzz": "bar"})
    # A dotted key whose head is a plain field is also rejected.
    with pytest.raises(ValueError, match="Key 'c.x' does not correspond"):
        configure(Grandpa(), {"c.x": 1})


def test_only_component_instances_can_be_configured():
    class Plain:
        a: int = Field()

    @component
    class Comp:
        b: int = Field()

    class Undecorated(Comp):
        c: int = Field()

    for target in (Plain(), Comp, Undecorated()):
        with pytest.raises(
            TypeError, match="Only @component, @factory, and @task instances can be configured."
        ):
            configure(target, {"b": 3})


def test_configure_only_once():
    p = make_pair()()
    configure(p, {"left": 1})
    with pytest.raises(ValueError, match="has already been configured"):
        configure(p, {"left": 2})


# --- allow_missing (component_test.py:575-646) ----------------------------- #


def test_allow_missing_plain_field():
    @component
    class A:
        a: int = Field()
        b: float = Field(allow_missing=True)

        @Field
        def c(self) -> float:
            return self.b if hasattr(self, "b") else self.a

    with pytest.raises(
        ValueError, match="No configuration value found for annotated field 'A.a' of type 'int'."
    ):
        configure(A(), {"b": 3.14})
    x = A()
    configure(x, {"a": 0})
    assert x.c == 0
    x = A()
    configure(x, {"a": 0, "b": 3.14})
    assert x.c == 3.14


def test_allow_missing_component_field():
    class Base:
        a: int = Field()

    @component
    class K1(Base):
        a = Field(5)

    @component
    class K2(Base):
        a = Field(5)

    @component
    class Holder:
        kid: Base = ComponentField()
        optional_kid: Base = ComponentField(allow_missing=True)

    with pytest.raises(
        ValueError,
        match="Component field 'Holder.kid' of type 'Base' has no default or configured class.",
    ):
        configure(Holder(), {"optional_kid": "K2"})
    h = Holder()
    configure(h, {"kid": "K1"})
    assert not hasattr(h, "optional_kid")


def test_allow_missing_field_still_inherits():
    @component
    class Kid:
        a: int = Field(allow_missing=True)

    @component
    class Dad:
        a: int = Field(5)
        kid: Kid = ComponentField(Kid)

    d = Dad()
    configure(d, {})
    assert d.kid.a == 5


# --- mutation guards (component_test.py:649-670) --------------------------- #


def test_setattr_before_and_after_configure():
    @component
    class A:
        a: int = Field(6)
        b: float = Field(allow_missing=True)

    x = A()
    x.a = 3
    x.b = 5.0
    configure(x, {"a": 0})
    assert (x.a, x.b) == (0, 5.0)
    with pytest.raises(
        ValueError,
        match="Setting already configured component field values directly is prohibited.",
    ):
        x.a = 5


def test_delete_is_prohibited_and_dir_lists_fields():
    p = make_pair()(left=1)
    with pytest.raises(ValueError, match="Deleting component field values is prohibited."):
        del p.left
    assert {"left", "right"} <= set(dir(p))


def test_cached_field_read_is_plain_attribute():
    """Design property: once resolved, a field lives in the instance dict."""
    p = make_pair()()
    configure(p, {"left": 3})
    assert p.left == 3
    assert p.__dict__["left"] == 3
