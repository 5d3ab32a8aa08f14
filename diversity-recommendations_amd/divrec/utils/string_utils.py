"""Metric names (reference divrec/utils/string_utils.py:1-7): a class name in
CamelCase becomes snake_case, an underscore inserted before each capital that
starts a lower-case run ("IntraListDiversityScore" -> "intra_list_diversity_score")."""


def to_camel_case(s: str) -> str:
    out = [s[0].lower()]
    for prev_i in range(1, len(s) - 1):
        ch, nxt = s[prev_i], s[prev_i + 1]
        if ch.isupper() and nxt.islower():
            out.append("_")
        out.append(ch.lower())
    out.append(s[-1].lower())
    return "".join(out)
