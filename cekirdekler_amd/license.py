"""License accessor (reference ``License.cs:58`` prints the GPL notice
because the library has no UI)."""

NOTICE = """cekirdekler_amd: an MI355X-native multi-device compute runtime with the
capabilities of Cekirdekler (C# explicit multi-device load-balancer OpenCL
wrapper, Copyright (C) 2017 Huseyin Tugrul BUYUKISIK, GPL-3.0-or-later).

This program is free software: you can redistribute it and/or modify it under
the terms of the GNU General Public License as published by the Free Software
Foundation, either version 3 of the License, or (at your option) any later
version.  This program is distributed in the hope that it will be useful, but
WITHOUT ANY WARRANTY; without even the implied warranty of MERCHANTABILITY or
FITNESS FOR A PARTICULAR PURPOSE.  See the GNU General Public License for more
details: <https://www.gnu.org/licenses/>."""


def license_text() -> str:
    return NOTICE
