"""The global click command group and the ``key=value`` parameter type.

Parity: zookeeper/core/cli.py:8-58 — ``key=value`` tokens (exactly one ``=``,
keys matching ``^[\\w.]+$``), ``--flag`` → True and ``--no-flag`` → False,
literal-eval'd values with a string fallback, exit code 2 on a malformed
token, and snake-case-insensitive command lookup (``TrainImageNet`` ≡
``train_image_net`` ≡ ``trainImageNet``).
"""

from __future__ import annotations

import re
from typing import Any, Optional, Tuple

import click

from zookeeper_amd.core.utils import convert_to_snake_case, parse_value_from_string

_KEY = re.compile(r"^[\w.]+$")
_TRUE_FLAG = re.compile(r"^--[\w.]+$")
_FALSE_FLAG = re.compile(r"^--no-[\w.]+$")


class ConfigParam(click.ParamType):
    """Converts one CLI token into a ``(key, value)`` pair."""

    name = "key=value"

    def convert(self, value: Any, param: Optional[click.Parameter], ctx) -> Tuple[str, Any]:
        if isinstance(value, tuple):  # already converted (e.g. default values)
            return value
        token = str(value)
        if _FALSE_FLAG.match(token):
            return token[len("--no-"):], False
        if _TRUE_FLAG.match(token):
            return token[2:], True

        parts = token.split("=")
        if len(parts) != 2 or not _KEY.match(parts[0]):
            self.fail(
                "configuration parameters must be of the form 'key=value', where "
                "the key contains only alpha-numeric characters, '_', and '.', "
                f"and the value doesn't contain '='. Received '{token}'.",
                param,
                ctx,
            )
        key, raw = parts
        try:
            parsed = parse_value_from_string(raw)
        except Exception:
            self.fail(
                f"unable to parse value of configuration parameter {token}. The "
                "only supported types are `int`, `float`, `str`, `None`, and "
                "lists/tuples of the above.",
                param,
                ctx,
            )
        return key, parsed


class CamelCaseGroup(click.Group):
    """Resolve a command by its snake-case form."""

    def get_command(self, ctx: click.Context, cmd_name: str):
        wanted = convert_to_snake_case(cmd_name)
        for registered in self.list_commands(ctx):
            if convert_to_snake_case(registered) == wanted:
                return super().get_command(ctx, registered)
        return None


@click.group(cls=CamelCaseGroup)
def cli() -> None:
    """Run a registered @task: ``<script> TaskName key=value ...``."""
